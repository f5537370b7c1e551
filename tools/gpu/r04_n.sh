#!/bin/bash
# round 4, call n: the host-trace run after a resident run, with more hardware queues per process
# (GPU_MAX_HW_QUEUES: with 4, the copy stream may share a queue with a prover stream)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
for q in 4 8 16; do
  echo "== GPU_MAX_HW_QUEUES=$q, warm-up resident" >> $O/r04n_queues.txt
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python3 -u tools/h2d_order.py resident,pipelined,resident,pipelined 0 10 resident >> $O/r04n_queues.txt 2>&1 || { tail -20 $O/r04n_queues.txt; exit 1; }
done
grep -v amdgpu.ids $O/r04n_queues.txt
