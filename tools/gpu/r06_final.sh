# Round 6 final validation: the driver's commands (-m gpu suite, smoke(), default bench line), then a rocprofv3
# kernel trace of the main leg whose k_hash_leaves durations are checked against that run's roofline.avg_ms.
# Outputs gpurun_out/r06_<tag>_*
set -e
TAG=${1:-final}
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu/r06_suite.sh $TAG
bash tools/gpu/r06_bench.sh $TAG
cd /tmp && export TMPDIR=/tmp
D=$R/gpurun_out/r06_${TAG}_ktrace
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline > $D.json 2> $D.err || { tail -20 $D.err; exit 1; }
find $D -name "*kernel_stats.csv" -exec cp {} $D.stats.csv \;
find $D -name "*kernel_trace.csv" -exec cp {} $D.trace.csv \;
python3 - $D <<'PY'
import csv, json, sys
d = sys.argv[1]
rows = [r for r in csv.DictReader(open(d + ".trace.csv")) if "k_hash_leaves" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
big = max(int(r["Grid_Size_X"]) for r in rows)  # the 2^23-row launches (one thread per LDE row)
last = [r for r in rows if int(r["Grid_Size_X"]) == big][-9:]  # the serial profiled region: 3 proofs x 3 commits
ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in last]
line = json.loads(open(d + ".json").read().strip().splitlines()[-1])
out = (f"# k_hash_leaves, the last 9 2^23-row launches of the traced run (the serial profiled region): "
       + " ".join(f"{x:.3f}" for x in ms) + f" ms\n# their mean {sum(ms) / len(ms):.4f} ms; the line's roofline.avg_ms "
       f"in the same run {line['roofline']['avg_ms']} ms ({line['roofline']['kernel']}, {line['roofline']['launches']} launches)\n")
open(d + ".check.txt", "w").write(out)
print(out)
PY
