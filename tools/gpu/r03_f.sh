#!/bin/bash
# round 3: FRI commit-phase timeline, LogUp register-cap sweep, bench with the SQ counter pass
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu/fri_timeline.sh r03f || exit $?
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/perm_waves_sweep.sh || exit $?
timeout -k 10 400 python3 bench.py --no-cpu-baseline > gpurun_out/r03f_bench.json 2> gpurun_out/r03f_bench.err
