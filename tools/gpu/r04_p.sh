#!/bin/bash
# round 4, call p: LogUp kernel A/B - the batches split into 2 or 3 inversion groups (LDS 40 / 32 KB per
# workgroup, 3 or 4 waves per SIMD) vs the default (one inversion, 80 KB, 2 waves) - and the opening dot
# products with register weights
# (default) vs the LDS weight table (ZKM_OPEN_LDS_WEIGHTS=1); shard bench only, kernel-trace stats of each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python3 -u -m pytest tests/test_compress_verify.py tests/test_compress_tree.py tests/test_gpu_prover.py -m gpu -v --timeout 600 --timeout-method thread > $O/r04p_gpu_tests.log 2>&1 || { tail -40 $O/r04p_gpu_tests.log; exit 1; }
tail -2 $O/r04p_gpu_tests.log
timeout -k 10 600 python3 -u tools/compress_node_timing.py > $O/r04p_node_timing.txt 2>&1 || { tail -20 $O/r04p_node_timing.txt; exit 1; }
grep -E "witness|node program" $O/r04p_node_timing.txt
ARGS="--steps 8 --warmup 2 --no-cpu-baseline --no-maxshape --no-compress --no-tendermint --no-sizes --no-pmc"
for v in "base:" "s2w3:ZKM_JIT_PERM_LDS_SPLIT=2 ZKM_JIT_PERM_WAVES=3" "s2w4:ZKM_JIT_PERM_LDS_SPLIT=2 ZKM_JIT_PERM_WAVES=4" "openlds:ZKM_OPEN_LDS_WEIGHTS=1" "s3w4:ZKM_JIT_PERM_LDS_SPLIT=3 ZKM_JIT_PERM_WAVES=4" "base2:"; do
  tag=${v%%:*}
  echo "== $tag"
  env ${v#*:} timeout -k 10 300 python3 -u bench.py $ARGS > $O/r04p_$tag.json 2> $O/r04p_$tag.err || { tail -20 $O/r04p_$tag.err; exit 1; }
  python3 -c "
import json
d = json.loads(open('$O/r04p_$tag.json').read().strip().splitlines()[-1])
def find(x, k):
    if isinstance(x, dict):
        if k in x: return x[k]
        for v in x.values():
            r = find(v, k)
            if r is not None: return r
st = find(d, 'stages_ms_per_shard') or {}
print('$tag', d['ms_per_step'], st.get('perm_trace'), st.get('open_eval'))"
done
ZKM_OPEN_LDS_WEIGHTS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r04p_prof1 -o run -- python3 bench.py $ARGS > $O/r04p_prof1.log 2>&1 || { tail -20 $O/r04p_prof1.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r04p_prof0 -o run -- python3 bench.py $ARGS > $O/r04p_prof0.log 2>&1 || { tail -20 $O/r04p_prof0.log; exit 1; }
for d in $O/r04p_prof0 $O/r04p_prof1; do f=$(find $d -name '*kernel_stats.csv' | head -1); echo "$d"; grep -E "perm|open|Name" "$f" | cut -c1-200; done
