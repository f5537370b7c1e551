# tests + bench at 1/2/3 shards in flight: bash tools/gpu/inflight2.sh <tag>
set -e
TAG=${1:-x}
mkdir -p gpurun_out
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t_$TAG.log 2>&1 || { tail -40 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
for k in 1 2 3; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --steps 4 --inflight $k > gpurun_out/bench_${TAG}_$k.json 2> gpurun_out/bench_${TAG}_$k.err || { tail -30 gpurun_out/bench_${TAG}_$k.err; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/bench_${TAG}_$k.json')); s=d['stages_ms_per_shard']
print('inflight $k: %.4g rows/s, %.2f ms/shard'%(d['value'], d['ms_per_shard']), {k: v['ms_per_shard'] for k, v in s.items() if not k.startswith('host')})"
done
