# Poseidon2 A/B + VALU probe + GPU tests + bench: bash tools/gpu/p2_ab.sh <tag>
set -e
TAG=${1:-x}
mkdir -p gpurun_out
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 120 tools/probe/valu_probe > gpurun_out/valu_$TAG.txt 2>&1
timeout -k 10 120 tools/probe/p2_probe > gpurun_out/p2ab_$TAG.txt 2>&1
cat gpurun_out/p2ab_$TAG.txt
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -2 gpurun_out/t_$TAG.log
timeout -k 10 600 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-400 gpurun_out/bench_$TAG.json
