# LDE kernel check + per-kernel timing: bash gpurun_ltest.sh <tag>
set -e
TAG=${1:-x}
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/lt_$TAG.log 2>&1 || { tail -30 gpurun_out/lt_$TAG.log; exit 1; }
tail -1 gpurun_out/lt_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/lde_$TAG -o run -- python3 -c "
import sys; sys.path.insert(0,'$R')
from zkmips_amd._lib import Device
d=Device(0)
for lg,w in [(22,67)]:
    ms=d.bench_lde(1<<lg,w,5); print('lde 2^%d x %d: %.2f ms'%(lg,w,ms))
" > $R/gpurun_out/lde_$TAG.log 2>&1
grep "lde 2" $R/gpurun_out/lde_$TAG.log
