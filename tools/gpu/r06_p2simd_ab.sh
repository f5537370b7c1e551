# Round 6: compress legs with the AVX-512 host Poseidon2 (B, libzkm_trace.so) vs the one-state code (A,
# libzkm_trace_a.so swapped in on this scratch copy), alternated, fresh process each; then the witness profile.
set -e
mkdir -p gpurun_out
cp zkmips_amd/libzkm_trace.so zkmips_amd/libzkm_trace_b.so
ARGS="--steps 2 --warmup 1 --no-maxshape --no-tendermint --no-sizes --no-pmc --no-cpu-baseline"
for i in 1 2; do
  for v in A B; do
    cp zkmips_amd/libzkm_trace_$(echo $v | tr AB ab).so zkmips_amd/libzkm_trace.so
    timeout -k 10 420 python -u bench.py $ARGS > gpurun_out/r06_p2s_${v}${i}.json 2> gpurun_out/r06_p2s_${v}${i}.err || { tail -30 gpurun_out/r06_p2s_${v}${i}.err; exit 1; }
    python3 - gpurun_out/r06_p2s_${v}${i}.json $v$i <<'PY'
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
cp zkmips_amd/libzkm_trace_b.so zkmips_amd/libzkm_trace.so
timeout -k 10 400 python -u tools/gpu/r06_wit_profile.py 16 > gpurun_out/r06_witprof16.txt 2>&1
