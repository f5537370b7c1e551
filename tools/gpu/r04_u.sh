#!/bin/bash
# round 4, call u: the device tracegen bench (now with every precompile chip) and its kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 400 python3 -u bench.py --workload tracegen --log-n 22 --steps 10 --warmup 2 > $O/r04u_tracegen.json 2> $O/r04u_tracegen.err || { tail -40 $O/r04u_tracegen.err; exit 1; }
tail -c 400 $O/r04u_tracegen.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/r04u_prof -o tg -- python3 -u bench.py --workload tracegen --log-n 22 --steps 10 --warmup 2 > $O/r04u_prof.log 2>&1 || { tail -40 $O/r04u_prof.log; exit 1; }
find $O/r04u_prof -name "*kernel_stats.csv" | head -3
