#!/bin/bash
# round 5, call l: calls j (openings A/B, cheaper weights) and k (LDE tiled A/B) in one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/r05_j.sh && bash tools/gpu/r05_k.sh
