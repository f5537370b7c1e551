#!/bin/bash
# round 5, call aq: openings' prefetching dot-product kernel walking 2 columns per block (ZKM_OPEN_CB=2, kind 3:
# 116 VGPRs, 4 waves per SIMD) vs 4 (154 VGPRs, 3 waves): prover / opening parity with 2, headline bench alternated
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
ZKM_OPEN_CB=2 timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_prover.py tests/test_blowup.py tests/test_gpu_kernels.py -m gpu > $O/r05aq_tests.log 2>&1 || { tail -40 $O/r05aq_tests.log; exit 1; }
echo "OPEN_CB=2: $(tail -1 $O/r05aq_tests.log)"
B="--steps 8 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline"
for i in 1 2 3; do
  for C in 4 2; do
    ZKM_OPEN_CB=$C timeout -k 10 300 python3 -u bench.py $B > $O/r05aq_c$C-$i.json 2> $O/r05aq_c$C-$i.err || { tail -20 $O/r05aq_c$C-$i.err; exit 1; }
  done
done
python3 - <<PY
import json
for C in (4, 2):
    for i in (1, 2, 3):
        d = json.loads(open("$O/r05aq_c%d-%d.json" % (C, i)).read().strip().splitlines()[-1])
        st = d["stages_ms_per_shard"]
        print("open_cb", C, i, "host-fed %.3f" % d["ms_per_shard"], "resident %.3f" % d["resident"]["ms_per_shard"],
              "open_eval %.3f" % st["open_eval"]["ms_per_shard"], "fri_reduce %.3f" % st["fri_reduce"]["ms_per_shard"])
PY
