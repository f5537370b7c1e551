# grouped openings: full GPU suite (byte parity) + core bench + core kernel trace + compress bench
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests_grouped.log 2>&1 || { tail -30 gpurun_out/r02_gpu_tests_grouped.log; exit 1; }
tail -1 gpurun_out/r02_gpu_tests_grouped.log
bash tools/gpu/core_prof.sh
timeout -k 10 400 python3 -u bench.py --workload compress --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r02_bench_compress_grouped.json 2> gpurun_out/r02_bench_compress_grouped.err || { tail -20 gpurun_out/r02_bench_compress_grouped.err; exit 1; }
cut -c1-200 gpurun_out/r02_bench_compress_grouped.json
