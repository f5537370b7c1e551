#!/bin/bash
# round 5, call ai: FRI reduced openings with 4 / 2 / 1 column loads in flight per thread (ZKM_RED_LOADS; call ah:
# 4 beat 8, 0.95 vs 1.125 ms per shard): prover byte parity with 2 and 1, then the headline bench alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
for L in 2 1; do
  ZKM_RED_LOADS=$L timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_prover.py -m gpu -k "bytes_identical" > $O/r05ai_tests$L.log 2>&1 || { tail -40 $O/r05ai_tests$L.log; exit 1; }
  echo "RED_LOADS=$L: $(tail -1 $O/r05ai_tests$L.log)"
done
B="--steps 8 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline"
for i in 1 2 3; do
  for L in 4 2 1; do
    ZKM_RED_LOADS=$L timeout -k 10 300 python3 -u bench.py $B > $O/r05ai_l$L-$i.json 2> $O/r05ai_l$L-$i.err || { tail -20 $O/r05ai_l$L-$i.err; exit 1; }
  done
done
python3 - <<PY
import json
for L in (4, 2, 1):
    for i in (1, 2, 3):
        d = json.loads(open("$O/r05ai_l%d-%d.json" % (L, i)).read().strip().splitlines()[-1])
        st = d["stages_ms_per_shard"]
        print("loads", L, i, "host-fed %.3f" % d["ms_per_shard"], "resident %.3f" % d["resident"]["ms_per_shard"],
              "fri_reduce %.3f" % st["fri_reduce"]["ms_per_shard"], "open_eval %.3f" % st["open_eval"]["ms_per_shard"],
              "lde %.3f" % st["lde"]["ms_per_shard"])
PY
