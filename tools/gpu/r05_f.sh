#!/bin/bash
# round 5, call f: the Poseidon2 probe again (VGPR-form MFMA; layer and whole-permutation A/B, exact outputs
# compared) with both SQ counter passes kept apart
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/probe/p2_mfma_probe > $O/r05f_p2_mfma.txt 2>&1 || { cat $O/r05f_p2_mfma.txt; exit 1; }
cat $O/r05f_p2_mfma.txt
cd /tmp
i=0
for C in "SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/r05f_pmc$i -o p2 -- $R/tools/probe/p2_mfma_probe 1024 > $O/r05f_pmc$i.log 2>&1 || { tail -20 $O/r05f_pmc$i.log; exit 1; }
done
cd $R
find $O/r05f_pmc1 $O/r05f_pmc2 -name "*counter_collection.csv"
