#!/bin/bash
# round 5, call t: calls r (suite, smoke, default line) and s (kernel-trace check) on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/r05_r.sh && bash tools/gpu/r05_s.sh
