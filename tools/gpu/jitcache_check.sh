# in-process JIT kernel cache: full GPU suite + compress setup time
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r02_gpu_tests_jitcache.log 2>&1 || { tail -30 gpurun_out/r02_gpu_tests_jitcache.log; exit 1; }
tail -1 gpurun_out/r02_gpu_tests_jitcache.log
bash tools/gpu/compress_setup.sh
