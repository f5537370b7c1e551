#!/bin/bash
# round 4, call l: does a resident run earlier in the process slow the host-trace runs after it? And the
# strided-tile access-pattern probe (tools/probe/tile_probe.hip)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 120 tools/probe/tile_probe > $O/r04l_tile_probe.txt 2>&1 || { cat $O/r04l_tile_probe.txt; exit 1; }
cat $O/r04l_tile_probe.txt
for spec in "pipelined,pipelined 0 10 pipelined" "pipelined,pipelined 0 10 resident" "pipelined,pipelined 0 10 per_call"; do
  echo "== $spec" >> $O/r04l_order.txt
  timeout -k 10 400 python3 -u tools/h2d_order.py $spec >> $O/r04l_order.txt 2>&1 || { tail -20 $O/r04l_order.txt; exit 1; }
done
echo "== DMA probe (copies as pipelined, proofs from the resident traces), warm-up resident" >> $O/r04l_order.txt
ZKM_BENCH_DMA_PROBE=1 timeout -k 10 400 python3 -u tools/h2d_order.py pipelined,pipelined 0 10 resident >> $O/r04l_order.txt 2>&1 || { tail -20 $O/r04l_order.txt; exit 1; }
grep -v amdgpu.ids $O/r04l_order.txt
