#!/bin/bash
# round 4, call f: the PCIe ceiling of the host-trace mode (pure H2D copy rates of one shard's trace bytes)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python3 -u tools/h2d_rate.py > $O/r04f_h2d_rate.txt 2>&1 || { tail -30 $O/r04f_h2d_rate.txt; exit 1; }
cat $O/r04f_h2d_rate.txt
