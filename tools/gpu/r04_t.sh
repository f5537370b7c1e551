#!/bin/bash
# round 4, call t: the KeccakSponge device trace, then the whole GPU suite, smoke and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_tracegen.py -m gpu -k keccak -v --timeout 240 --timeout-method thread > $O/r04t_keccak.log 2>&1 || { tail -60 $O/r04t_keccak.log; exit 1; }
tail -3 $O/r04t_keccak.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r04t_gpu_tests.log 2>&1 || { tail -60 $O/r04t_gpu_tests.log; exit 1; }
tail -3 $O/r04t_gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r04t_smoke.log 2>&1 || { tail -40 $O/r04t_smoke.log; exit 1; }
tail -2 $O/r04t_smoke.log
