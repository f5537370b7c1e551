# Round 6: column-batch size of the LDE (ZKM_LDE_CB = columns per batch), fresh process each: ms per LDE of
# 2^23 x 64, 2^23 x 44, 2^22 x 64, 2^21 x 67
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  for cb in 2 4 8 16; do
    ZKM_LDE_CB=$cb timeout -k 10 120 python -c "
import sys; sys.path.insert(0, '.')
from zkmips_amd._lib import Device
d = Device(0)
print('cb $cb', ' '.join('%.4f' % d.bench_lde(1 << L, W, 10) for L, W in [(23, 64), (23, 44), (22, 64), (21, 67)]), flush=True)"
  done
done
