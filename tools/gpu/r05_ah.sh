#!/bin/bash
# round 5, call ah: FRI reduced openings with 4 column loads in flight per thread (ZKM_RED_LOADS=4) vs 8; (call ag: 16 loads, 72 VGPRs, 7 waves
# per SIMD) vs 8 (52 VGPRs, 8 waves): prover byte parity with 16, then the headline bench alternated (stage table)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
ZKM_RED_LOADS=4 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_prover.py tests/test_blowup.py -m gpu > $O/r05ah_tests.log 2>&1 || { tail -40 $O/r05ah_tests.log; exit 1; }
echo "RED_LOADS=4: $(tail -1 $O/r05ah_tests.log)"
B="--steps 8 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline"
for i in 1 2 3; do
  for L in 8 4; do
    ZKM_RED_LOADS=$L timeout -k 10 300 python3 -u bench.py $B > $O/r05ah_l$L-$i.json 2> $O/r05ah_l$L-$i.err || { tail -20 $O/r05ah_l$L-$i.err; exit 1; }
  done
done
python3 - <<PY
import json
for L in (8, 4):
    for i in (1, 2, 3):
        d = json.loads(open("$O/r05ah_l%d-%d.json" % (L, i)).read().strip().splitlines()[-1])
        st = d["stages_ms_per_shard"]
        print("loads", L, i, "host-fed %.3f" % d["ms_per_shard"], "resident %.3f" % d["resident"]["ms_per_shard"],
              "fri_reduce %.3f" % st["fri_reduce"]["ms_per_shard"], "open_eval %.3f" % st["open_eval"]["ms_per_shard"],
              "lde %.3f" % st["lde"]["ms_per_shard"])
PY
