#!/bin/bash
# round 4, call k: is the bench's host-trace run slow because it follows the resident run (order / clocks)?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for spec in "resident,pipelined,resident,pipelined 0" "pipelined,resident,pipelined,resident 0" "resident,pipelined,resident,pipelined 5"; do
  echo "== $spec" >> $O/r04k_order.txt
  timeout -k 10 400 python3 -u tools/h2d_order.py $spec >> $O/r04k_order.txt 2>&1 || { tail -20 $O/r04k_order.txt; exit 1; }
done
grep -v amdgpu.ids $O/r04k_order.txt
