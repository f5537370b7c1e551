#!/bin/bash
# round 4, call i: shards in flight 2/3/4/5 (resident and host traces), then the default bench line with the
# tendermint traces generated after the timed regions
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for k in 3 4 2 5 3 4; do
  timeout -k 10 300 python3 -u tools/h2d_attrib.py resident 8 22 $k >> $O/r04i_inflight.txt 2>&1 || { tail -20 $O/r04i_inflight.txt; exit 1; }
done
for k in 3 4; do
  timeout -k 10 300 python3 -u tools/h2d_attrib.py pipelined 8 22 $k >> $O/r04i_inflight.txt 2>&1 || { tail -20 $O/r04i_inflight.txt; exit 1; }
done
grep -v amdgpu.ids $O/r04i_inflight.txt | cut -c1-120
timeout -k 10 900 python3 -u bench.py --steps 10 --warmup 2 > $O/r04i_bench.log 2>&1 || { tail -30 $O/r04i_bench.log; exit 1; }
tail -1 $O/r04i_bench.log | cut -c1-300
