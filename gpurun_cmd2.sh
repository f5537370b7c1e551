set -e
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_prover.py -x -q > gpurun_out/t2.log 2>&1 || { tail -60 gpurun_out/t2.log; exit 1; }
tail -3 gpurun_out/t2.log
