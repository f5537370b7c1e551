# Round 6: optional pytest selection (PYTEST_K) then the default bench line; outputs gpurun_out/r06_<tag>_*
set -e
TAG=${1:-a}
shift || true
mkdir -p gpurun_out
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$PYTEST_K" --timeout 600 --timeout-method thread > gpurun_out/r06_${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/r06_${TAG}_tests.log; exit 1; }
  tail -3 gpurun_out/r06_${TAG}_tests.log
fi
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/r06_${TAG}_bench.json 2> gpurun_out/r06_${TAG}_bench.err || { tail -40 gpurun_out/r06_${TAG}_bench.err; exit 1; }
python3 - "$TAG" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r06_{sys.argv[1]}_bench.json").read().strip().splitlines()[-1])
print("value", d["value"], "ms_per_step", d["ms_per_step"])
for k in ("resident", "host_traces", "stages", "sizes", "ntt", "roofline"):
    if k in d: print(k, json.dumps(d[k])[:900])
PY
