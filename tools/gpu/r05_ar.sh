#!/bin/bash
# round 5, call ar: the driver's commands on HEAD (openings 2 columns per block) -- the whole -m gpu
# suite, smoke(), the default bench line -- then the kernel-trace summary of the headline workload checked against
# the line's roofline.avg_ms
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 1200 python3 -u -m pytest tests/ -x -v -m gpu --timeout 600 --timeout-method thread --durations=15 > $O/r05ar_gpu_tests.log 2>&1 || { tail -60 $O/r05ar_gpu_tests.log; exit 1; }
tail -3 $O/r05ar_gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r05ar_smoke.log 2>&1 || { tail -30 $O/r05ar_smoke.log; exit 1; }
tail -1 $O/r05ar_smoke.log
timeout -k 10 1200 python3 -u bench.py > $O/r05ar_bench.json 2> $O/r05ar_bench.err || { tail -40 $O/r05ar_bench.err; exit 1; }
tail -c 600 $O/r05ar_bench.json
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05ar_prof -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline > $O/r05ar_prof_bench.json 2> $O/r05ar_prof.err || { tail -20 $O/r05ar_prof.err; exit 1; }
find $O/r05ar_prof -name "*kernel_stats.csv" -exec cp {} $O/r05ar_kernel_stats.csv \;
find $O/r05ar_prof -name "*kernel_trace.csv" -exec cp {} $O/r05ar_kernel_trace.csv \;
cd $R
python3 - > $O/r05ar_kernel_trace_check.txt <<PY
import csv, json
rows = []
for r in csv.DictReader(open("$O/r05ar_kernel_trace.csv")):
    if "k_hash_leaves" in r["Kernel_Name"]:
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Grid_Size_X"])))
rows.sort()
big = [r for r in rows if r[2] >= (1 << 23)]
last = big[-9:]
ms = [(e - s) / 1e6 for s, e, _ in last]
d = json.loads(open("$O/r05ar_prof_bench.json").read().strip().splitlines()[-1])
print("# rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 5 --warmup 1 --no-pmc --no-sizes --no-maxshape")
print("#   --no-compress --no-tendermint --no-cpu-baseline  (tools/gpu/r05_ar.sh); summary r05_kernel_stats_final.csv")
print("# the 2^23-row k_hash_leaves launches of the serial profiled region (3 proofs x main / perm / quotient commit):")
print("  " + " ".join("%.3f" % x for x in ms) + " ms")
print("# their mean: %.4f ms; the line's roofline.avg_ms in the same run: %.4f ms (kernel %s, %d launches)"
      % (sum(ms) / len(ms), d["roofline"]["avg_ms"], d["roofline"]["kernel"], d["roofline"]["launches"]))
PY
cat $O/r05ar_kernel_trace_check.txt
