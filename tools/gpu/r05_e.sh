#!/bin/bash
# round 5, call e: (1) the Poseidon2 external-layer probe (64-bit VALU / 32-bit VALU / i8 MFMA forms; exact
# outputs compared), its SQ counters; (2) the LDE microbench's kernel breakdown; (3) the CPU-share probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/probe/p2_mfma_probe > $O/r05e_p2_mfma.txt 2>&1 || { cat $O/r05e_p2_mfma.txt; exit 1; }
cat $O/r05e_p2_mfma.txt
cat > /tmp/lde1.py <<PY
import os, sys
sys.path.insert(0, os.environ['GRAFT_REPO_ROOT'])
from zkmips_amd._lib import Device
d = Device(0)
d.bench_lde(1 << 22, 67, 2)
print('lde 2^22x67 %.3f ms' % d.bench_lde(1 << 22, 67, 5), flush=True)
PY
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05e_lde -o lde -- python3 /tmp/lde1.py > $O/r05e_lde.log 2>&1 || { tail -20 $O/r05e_lde.log; exit 1; }
find $O/r05e_lde -name "*kernel_stats.csv" -exec cp {} $O/r05e_lde_kernel_stats.csv \;
cd $R
timeout -k 10 600 python3 tools/cpu_cliff.py > $O/r05e_cpu_cliff.txt 2>&1 || { tail -20 $O/r05e_cpu_cliff.txt; exit 1; }
tail -12 $O/r05e_cpu_cliff.txt
cd /tmp
for C in "SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/r05e_pmc -o p2 -- $R/tools/probe/p2_mfma_probe 1024 > $O/r05e_pmc.log 2>&1 || { tail -20 $O/r05e_pmc.log; exit 1; }
done
cd $R
find $O/r05e_pmc -name "*counter_collection.csv" | head
