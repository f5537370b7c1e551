#!/bin/bash
# round 5, call ak: kernel-trace summary of the compress leg (64-leaf tree of recursion-machine proofs, config 5)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05ak_prof -o run -- python3 $R/bench.py --workload compress --steps 1 --warmup 1 --no-pmc --no-cpu-baseline > $O/r05ak_bench.json 2> $O/r05ak_bench.err || { tail -20 $O/r05ak_bench.err; exit 1; }
find $O/r05ak_prof -name "*kernel_stats.csv" -exec cp {} $O/r05ak_kernel_stats.csv \;
find $O/r05ak_prof -name "*kernel_trace.csv" -exec cp {} $O/r05ak_kernel_trace.csv \;
tail -c 1500 $O/r05ak_bench.json
python3 - <<PY
import csv
rows = list(csv.DictReader(open("$O/r05ak_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms %.1f, launches %d" % (tot / 1e6, sum(int(r["Calls"]) for r in rows)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print("%-60s %6s %9.1f us %5.1f %%" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3, 100 * float(r["TotalDurationNs"]) / tot))
PY
