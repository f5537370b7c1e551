# 2-rank rehearsal of the headline N>1 flow (NUMA bind + staggered copies) + the service GPU tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu/rehearse2.sh
timeout -k 10 300 python -u -m pytest tests/test_service.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r02_gpu_tests_service.log 2>&1 || { tail -30 gpurun_out/r02_gpu_tests_service.log; exit 1; }
tail -2 gpurun_out/r02_gpu_tests_service.log
