#!/bin/bash
# round 5, call h: (1) kernel-trace summary of the short fib line (resident + host + profiled proofs: the current
# per-kernel table for openings / FRI / Merkle); (2) the fib line with the maxshape leg (records mode with its
# per-step diagnostics, native record conversion)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05h_prof -o fib -- python3 $R/bench.py --steps 4 --no-cpu-baseline --no-maxshape --no-compress --no-tendermint --no-sizes --no-pmc > $O/r05h_prof.json 2> $O/r05h_prof.err || { tail -20 $O/r05h_prof.err; exit 1; }
find $O/r05h_prof -name "*kernel_stats.csv" -exec cp {} $O/r05h_kernel_stats.csv \;
cd $R
timeout -k 10 600 python3 bench.py --steps 4 --no-cpu-baseline --no-compress --no-tendermint --no-sizes --no-pmc > $O/r05h_maxshape.json 2> $O/r05h_maxshape.err || { tail -20 $O/r05h_maxshape.err; exit 1; }
python3 - <<PY
import json
d = json.loads(open("$O/r05h_maxshape.json").read().strip().splitlines()[-1])
m = d["maxshape"]
print(json.dumps({k: m[k] for k in m if k not in ("workload",)}, indent=1)[:3000])
PY
