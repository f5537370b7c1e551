#!/bin/bash
# round 5, call al: the host-fed headline's H2D copies ran as __amd_rocclr_copyBuffer blit kernels on the CUs in the
# round's kernel traces (65 launches of ~1.9 ms, 512-thread workgroups on every CU).  The box's SDMA settings, then
# the headline with HSA_ENABLE_SDMA=1 against the default, alternated; a kernel trace of the SDMA=1 run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
env | grep -i -E "sdma|blit|HSA_|HIP_|GPU_" | sort > $O/r05al_env.txt || true
cat $O/r05al_env.txt
B="--steps 8 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline"
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py $B > $O/r05al_def$i.json 2> $O/r05al_def$i.err || { tail -20 $O/r05al_def$i.err; exit 1; }
  HSA_ENABLE_SDMA=1 timeout -k 10 300 python3 -u bench.py $B > $O/r05al_sdma$i.json 2> $O/r05al_sdma$i.err || { tail -20 $O/r05al_sdma$i.err; exit 1; }
done
python3 - <<PY
import json
for v in ("def", "sdma"):
    for i in (1, 2):
        d = json.loads(open("$O/r05al_%s%d.json" % (v, i)).read().strip().splitlines()[-1])
        h = d["host_traces"]
        print(v, i, "host-fed %.3f" % d["ms_per_shard"], "resident %.3f" % d["resident"]["ms_per_shard"], "vs %.3f" % h["vs_resident"],
              "h2d alone %.2f ms %.1f GB/s" % (h["h2d_alone_ms_per_shard"], h["h2d_GBps"]), "waits", h["copy_wait_ms"])
PY
cd /tmp
HSA_ENABLE_SDMA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r05al_prof -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline > $O/r05al_prof.json 2> $O/r05al_prof.err || { tail -20 $O/r05al_prof.err; exit 1; }
f=$(find $O/r05al_prof -name "*kernel_stats.csv" | head -1)
grep -i copy "$f" || echo "no copy kernels with HSA_ENABLE_SDMA=1"
