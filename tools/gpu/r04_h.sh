#!/bin/bash
# round 4, call h: host-trace mode with one FIFO copy stream for all slots vs one stream per slot (A/B,
# alternating), then the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for i in 1 2; do
  for m in slot shared; do
    echo "copy streams: $m" >> $O/r04h_copy_ab.txt
    ZKM_BENCH_COPY_STREAMS=$m timeout -k 10 300 python3 -u tools/h2d_attrib.py pipelined 8 >> $O/r04h_copy_ab.txt 2>&1 || { tail -20 $O/r04h_copy_ab.txt; exit 1; }
  done
done
timeout -k 10 300 python3 -u tools/h2d_attrib.py resident 8 >> $O/r04h_copy_ab.txt 2>&1 || { tail -20 $O/r04h_copy_ab.txt; exit 1; }
grep -v amdgpu.ids $O/r04h_copy_ab.txt
timeout -k 10 900 python3 -u bench.py --steps 10 --warmup 2 > $O/r04h_bench.log 2>&1 || { tail -30 $O/r04h_bench.log; exit 1; }
tail -1 $O/r04h_bench.log | cut -c1-300
