#!/bin/bash
# round 5, call aj: JIT kernels' column-load lookahead (ZKM_JIT_LOOKAHEAD_Q for the quotient kernel, default 8;
# ZKM_JIT_LOOKAHEAD_P for the LogUp kernel, default 48), after fewer loads in flight won in the FRI reduction:
# headline bench alternated, quotient / perm_trace stage times; prover bytes with the two non-default extremes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
ZKM_JIT_LOOKAHEAD_Q=4 ZKM_JIT_LOOKAHEAD_P=24 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_prover.py -m gpu -k "bytes_identical" > $O/r05aj_tests.log 2>&1 || { tail -40 $O/r05aj_tests.log; exit 1; }
echo "Q4 P24: $(tail -1 $O/r05aj_tests.log)"
B="--steps 8 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline"
for i in 1 2; do
  for C in "8 48" "4 48" "12 48" "8 24" "8 96"; do
    set -- $C
    ZKM_JIT_LOOKAHEAD_Q=$1 ZKM_JIT_LOOKAHEAD_P=$2 timeout -k 10 300 python3 -u bench.py $B > $O/r05aj_q$1p$2-$i.json 2> $O/r05aj_q$1p$2-$i.err || { tail -20 $O/r05aj_q$1p$2-$i.err; exit 1; }
  done
done
python3 - <<PY
import json
for c in ("8 48", "4 48", "12 48", "8 24", "8 96"):
    q, p = c.split()
    for i in (1, 2):
        d = json.loads(open("$O/r05aj_q%sp%s-%d.json" % (q, p, i)).read().strip().splitlines()[-1])
        st = d["stages_ms_per_shard"]
        print("Q%s P%s" % (q, p), i, "host-fed %.3f" % d["ms_per_shard"], "resident %.3f" % d["resident"]["ms_per_shard"],
              "quotient %.3f" % st["quotient"]["ms_per_shard"], "perm_trace %.3f" % st["perm_trace"]["ms_per_shard"])
PY
