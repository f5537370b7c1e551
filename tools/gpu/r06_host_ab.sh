# Round 6: compress legs end to end, A = the package in ab_old/ (prepared by hand: an earlier commit, or the tree
# without the change under test) against the working tree (B), alternated, fresh process each.  gpurun_out/r06_<tag>_*
set -e
TAG=${1:-hab}
mkdir -p gpurun_out
ARGS="--steps 2 --warmup 1 --no-maxshape --no-tendermint --no-sizes --no-pmc --no-cpu-baseline"
for i in 1 2; do
  for v in A B; do
    if [ $v = A ]; then D=ab_old; else D=.; fi
    (cd $D && timeout -k 10 420 python -u bench.py $ARGS) > gpurun_out/r06_${TAG}_${v}${i}.json 2> gpurun_out/r06_${TAG}_${v}${i}.err || { tail -30 gpurun_out/r06_${TAG}_${v}${i}.err; exit 1; }
    python3 - gpurun_out/r06_${TAG}_${v}${i}.json $v$i <<'PY'
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
