# full GPU suite + compress bench line + smoke
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=10 > gpurun_out/r02_gpu_tests_full.log 2>&1 || { tail -30 gpurun_out/r02_gpu_tests_full.log; exit 1; }
tail -2 gpurun_out/r02_gpu_tests_full.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 || { tail -20 gpurun_out/r02_smoke.log; exit 1; }
tail -2 gpurun_out/r02_smoke.log
timeout -k 10 400 python3 -u bench.py --workload compress --steps 3 --warmup 1 > gpurun_out/r02_bench_compress.json 2> gpurun_out/r02_bench_compress.err || { tail -20 gpurun_out/r02_bench_compress.err; exit 1; }
cut -c1-300 gpurun_out/r02_bench_compress.json
