# LDE column-batch sweep + LDE tests + bench: bash tools/gpu/lde_cb.sh <tag>
set -e
TAG=${1:-x}
mkdir -p gpurun_out
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/lt_$TAG.log 2>&1 || { tail -30 gpurun_out/lt_$TAG.log; exit 1; }
tail -1 gpurun_out/lt_$TAG.log
for cb in 0 1 2 4 8 16; do
  ZKM_LDE_CB=$cb timeout -k 10 120 python3 -c "
import sys; sys.path.insert(0,'.')
from zkmips_amd._lib import Device
d=Device(0)
print('cb $cb lde 2^22 x 67: %.3f ms'%d.bench_lde(1<<22,67,5))
" 2>&1 | tail -1
done
timeout -k 10 600 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cut -c1-300 gpurun_out/bench_$TAG.json
