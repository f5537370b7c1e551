set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/t1.log 2>&1 || { tail -50 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 120 python -c "
from zkmips_amd._lib import Device
d=Device(0)
for lg,w in [(20,67),(22,67),(22,119)]:
    ms=d.bench_lde(1<<lg,w,5); n=1<<lg
    print('lde 2^%d x %d: %.2f ms  -> algorithmic %.1f GB/s'%(lg,w,ms, 12*n*w/ms/1e6))
" 2>&1 | tee gpurun_out/b1.log
