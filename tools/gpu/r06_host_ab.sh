# Round 6: compress legs end to end, the package at an earlier commit (A: ab_old/, prepared by hand with that
# commit's host library) against HEAD (B), alternated, fresh process each.  Outputs gpurun_out/r06_hab_*
set -e
mkdir -p gpurun_out
ARGS="--steps 2 --warmup 1 --no-maxshape --no-tendermint --no-sizes --no-pmc --no-cpu-baseline"
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then D=ab_old; else D=.; fi
    (cd $D && timeout -k 10 420 python -u bench.py $ARGS) > gpurun_out/r06_hab_${v}${i}.json 2> gpurun_out/r06_hab_${v}${i}.err || { tail -30 gpurun_out/r06_hab_${v}${i}.err; exit 1; }
    python3 - gpurun_out/r06_hab_${v}${i}.json $v$i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in ("compress", "compress_2e21"):
    c = d.get(k) or {}
    print(sys.argv[2], k, c.get("value"), "wall", c.get("tree_wall_s"), "prove_only", (c.get("prove_only") or {}).get("value"),
          "wit", c.get("witness_generation", {}).get("build_s_per_node"), c.get("witness_generation", {}).get("execute_and_traces_s_per_node"),
          "tl", json.dumps(c.get("timeline")), flush=True)
PY
  done
done
