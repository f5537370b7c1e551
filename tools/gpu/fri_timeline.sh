# kernel timeline of serial FibCpu 2^22 proofs (FRI commit phase gaps): bash tools/gpu/fri_timeline.sh <tag>
set -o pipefail
TAG=${1:-cur}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl_$TAG -o run -- python3 $R/tools/gpu/prove_serial.py 3 > $R/gpurun_out/tl_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/tl_$TAG.log; exit 1; }
find $R/gpurun_out/tl_$TAG -name "*kernel_trace.csv" -exec cp {} $R/gpurun_out/ktrace_$TAG.csv \;
