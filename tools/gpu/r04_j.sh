#!/bin/bash
# round 4, call j: host-trace mode with each slot's copies issued atomically on the shared FIFO stream; per-call
# proof times resident vs pipelined; then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for m in pipelined resident pipelined; do
  timeout -k 10 300 python3 -u tools/h2d_attrib.py $m 8 >> $O/r04j_attrib.txt 2>&1 || { tail -20 $O/r04j_attrib.txt; exit 1; }
done
grep -v amdgpu.ids $O/r04j_attrib.txt | cut -c1-220
timeout -k 10 900 python3 -u bench.py --steps 10 --warmup 2 > $O/r04j_bench.log 2>&1 || { tail -30 $O/r04j_bench.log; exit 1; }
tail -1 $O/r04j_bench.log | cut -c1-300
