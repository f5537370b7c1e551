#!/bin/bash
# round 5, call b: the default bench line on the SURVEY 8d basis (host traces headline, records-fed maxshape)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}"
timeout -k 10 900 python3 -u bench.py --steps 20 --warmup 2 > $O/r05b_bench.json 2> $O/r05b_bench.err || { tail -40 $O/r05b_bench.err; exit 1; }
tail -c 400 $O/r05b_bench.json
