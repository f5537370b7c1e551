# SQ counters over the LDE microbench: bash gpurun_pmc_lde.sh <tag>
set -e
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
cat > /tmp/ldeb.py <<PY
import sys; sys.path.insert(0,'$R')
from zkmips_amd._lib import Device
d=Device(0)
print('lde %.2f ms'%d.bench_lde(1<<22,67,2))
PY
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmcl_$TAG -o run -- python3 /tmp/ldeb.py > $R/gpurun_out/pmcl_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmcl2_$TAG -o run -- python3 /tmp/ldeb.py > $R/gpurun_out/pmcl2_$TAG.log 2>&1
echo done
