# 16-lane Poseidon2WideDeg3 trace kernel: parity tests + tracegen bench
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_recursion.py tests/test_tracegen.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_gpu_tests_p2trace.log 2>&1 || { tail -30 gpurun_out/r02_gpu_tests_p2trace.log; exit 1; }
tail -1 gpurun_out/r02_gpu_tests_p2trace.log
timeout -k 10 300 python -u bench.py --workload tracegen --steps 5 --warmup 1 > gpurun_out/r02_bench_tracegen.json 2> gpurun_out/r02_bench_tracegen.err || { tail -20 gpurun_out/r02_bench_tracegen.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r02_bench_tracegen.json').read().strip().splitlines()[-1]); print(d['chips']['Poseidon2WideDeg3'])"
