# recursion GPU tests (incl. the wide machine) + the k_compress_level look-ahead A/B
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_recursion.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests_wide.log 2>&1 || { tail -30 gpurun_out/r02_gpu_tests_wide.log; exit 1; }
tail -1 gpurun_out/r02_gpu_tests_wide.log
bash tools/gpu/cl_ab.sh
