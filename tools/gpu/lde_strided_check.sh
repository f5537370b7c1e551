# blowup-4 LDE written in place (no 2D copy): blowup/recursion/kernel parity + compress bench + kernel trace
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_blowup.py tests/test_recursion.py tests/test_gpu_kernels.py tests/test_gpu_prover.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests_lde4.log 2>&1 || { tail -30 gpurun_out/r02_gpu_tests_lde4.log; exit 1; }
tail -1 gpurun_out/r02_gpu_tests_lde4.log
timeout -k 10 400 python3 -u bench.py --workload compress --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02_bench_compress_lde4.json 2> gpurun_out/r02_bench_compress_lde4.err || { tail -20 gpurun_out/r02_bench_compress_lde4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r02_bench_compress_lde4.json').read().strip().splitlines()[-1]); print('compress', d['value'], d['ms_per_proof'], d['serial_ms_per_proof'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_compress -o run -- python3 $R/bench.py --workload compress --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline > $R/gpurun_out/prof_compress.log 2>&1 || { tail -20 $R/gpurun_out/prof_compress.log; exit 1; }
find $R/gpurun_out/prof_compress -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/kstats_compress.csv \;
