#!/bin/bash
# round 3 (session 2): kernel stats of the compress tree after the blowup-4 LDE change
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --workload compress --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline > gpurun_out/r03z_prof_compress.log 2>&1 || { tail -20 gpurun_out/r03z_prof_compress.log; exit 1; }
find gpurun_out/prof_c3 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r03z_kernel_stats_compress.csv
head -12 gpurun_out/r03z_kernel_stats_compress.csv | cut -c1-150
