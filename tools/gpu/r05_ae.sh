#!/bin/bash
# round 5, call ae: shard-level A/B of 8-column LDE batches with default-policy intermediate stores
# (libzkm_hip_ab.so -DZKM_LDE_MID_AUX=0, ZKM_LDE_CB=8) against the default (16 columns, non-temporal): the
# headline bench (resident + host-fed, stage table) alternated, three rounds
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
B="--steps 8 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py $B > $O/r05ae_base$i.json 2> $O/r05ae_base$i.err || { tail -20 $O/r05ae_base$i.err; exit 1; }
  ZKM_LIB=$R/zkmips_amd/libzkm_hip_ab.so ZKM_LDE_CB=8 timeout -k 10 300 python3 -u bench.py $B > $O/r05ae_mall$i.json 2> $O/r05ae_mall$i.err || { tail -20 $O/r05ae_mall$i.err; exit 1; }
done
python3 - <<PY
import json
for v in ("base", "mall"):
    for i in (1, 2, 3):
        d = json.loads(open("$O/r05ae_%s%d.json" % (v, i)).read().strip().splitlines()[-1])
        st = d["stages_ms_per_shard"]
        print(v, i, "host-fed %.3f ms" % d["ms_per_shard"], "resident %.3f ms" % d["resident"]["ms_per_shard"],
              "serial %.3f" % d["serial_ms_per_shard"], "lde %.3f" % st["lde"]["ms_per_shard"],
              "leaves %.3f" % st["merkle_leaves"]["ms_per_shard"])
PY
