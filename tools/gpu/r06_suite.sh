# Round 6: full -m gpu suite + smoke on the current tree (prebuilt libzkm_hip.so), logs under gpurun_out/r06_<tag>_*
set -e
TAG=${1:-a}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r06_${TAG}_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r06_${TAG}_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r06_${TAG}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_${TAG}_smoke.log 2>&1 || { tail -30 gpurun_out/r06_${TAG}_smoke.log; exit 1; }
cat gpurun_out/r06_${TAG}_smoke.log
