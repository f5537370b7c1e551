# full GPU suite + headline serial/pipelined + core + compress after removing per-chip host syncs
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests_sync.log 2>&1 || { tail -30 gpurun_out/r02_gpu_tests_sync.log; exit 1; }
tail -1 gpurun_out/r02_gpu_tests_sync.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/r02_bench_sync.json 2> gpurun_out/r02_bench_sync.err || { tail -20 gpurun_out/r02_bench_sync.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload core --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/r02_bench_core_sync.json 2> gpurun_out/r02_bench_core_sync.err || { tail -20 gpurun_out/r02_bench_core_sync.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --workload compress --steps 3 --warmup 1 > gpurun_out/r02_bench_compress_sync.json 2> gpurun_out/r02_bench_compress_sync.err || { tail -20 gpurun_out/r02_bench_compress_sync.err; exit 1; }
python3 - <<'PY'
import json
for f in ("r02_bench_sync", "r02_bench_core_sync"):
    d = json.loads(open(f"gpurun_out/{f}.json").read().strip().splitlines()[-1])
    print(f, "value", d["value"], "ms/shard", d["ms_per_shard"], "resident", d["resident"]["ms_per_shard"], "serial", d["serial_ms_per_shard"])
d = json.loads(open("gpurun_out/r02_bench_compress_sync.json").read().strip().splitlines()[-1])
print("compress", d["value"], d["ms_per_proof"], d["serial_ms_per_proof"], d["cpu_baseline"]["sample"])
PY
