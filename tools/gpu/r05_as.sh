#!/bin/bash
# round 5, call as: SQ counters over the LDE microbench (2^22 x 67) on the final kernels (sequential-coset fused
# tile, k_ntt_s9b), two counter passes, summed per kernel by tools/pmc_kernels.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
cat > /tmp/ldeb.py <<PY
import sys; sys.path.insert(0, '$R')
from zkmips_amd._lib import Device
d = Device(0)
print('lde %.3f ms' % d.bench_lde(1 << 22, 67, 2))
PY
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/r05as_pmc1 -o run -- python3 /tmp/ldeb.py > $O/r05as_pmc1.log 2>&1 || { tail -20 $O/r05as_pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/r05as_pmc2 -o run -- python3 /tmp/ldeb.py > $O/r05as_pmc2.log 2>&1 || { tail -20 $O/r05as_pmc2.log; exit 1; }
cd $R
python3 tools/pmc_kernels.py $O/r05as_pmc1 $O/r05as_pmc2 > $O/r05as_pmc.txt
head -80 $O/r05as_pmc.txt
