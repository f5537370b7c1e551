# Round 6: the 64-leaf compress tree (--workload compress) at 3 / 4 / 5 proofs in flight, alternated twice, fresh
# process each.  gpurun_out/r06_cif_<n><run>.json
set -e
mkdir -p gpurun_out
for run in 1 2; do
  for n in 3 4 5; do
    timeout -k 10 300 python -u bench.py --workload compress --no-cpu-baseline --inflight $n > gpurun_out/r06_cif_$n$run.json 2> gpurun_out/r06_cif_$n$run.err || { tail -30 gpurun_out/r06_cif_$n$run.err; exit 1; }
    python3 - gpurun_out/r06_cif_$n$run.json $n $run <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("inflight", sys.argv[2], "run", sys.argv[3], d["value"], "wall", d.get("tree_wall_s"), "prove_only", d.get("prove_only", {}).get("value"), flush=True)
PY
  done
done
