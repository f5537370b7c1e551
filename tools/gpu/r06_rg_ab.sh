# Round 6 A/B of the one-column-per-thread short strided passes (k_ntt_rg; B = in-tree build) against the previous build
# (A = zkmips_amd/libzkm_hip_a.so): LDE parity tests first, then the LDE microbench at 2^15..2^17 and the compress
# workload (prove-only rate), alternated twice, fresh process each.  gpurun_out/r06_rg_*
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_blowup.py -x -q -m gpu -k "lde or blowup or commit" --timeout 300 --timeout-method thread > gpurun_out/r06_rg_tests.log 2>&1 || { tail -30 gpurun_out/r06_rg_tests.log; exit 1; }
tail -2 gpurun_out/r06_rg_tests.log
CHILD="import sys; sys.path.insert(0, '$R'); from zkmips_amd._lib import Device; d = Device(0); print(' '.join('%.4f' % d.bench_lde(1 << L, W, 30) for L, W in [(15, 64), (16, 64), (17, 64), (16, 256), (17, 256)]))"
echo "LDE ms: 2^15x64 2^16x64 2^17x64 2^16x256 2^17x256"
for run in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export ZKM_LIB=$R/zkmips_amd/libzkm_hip_a.so; else unset ZKM_LIB; fi
    echo "$v$run $(timeout -k 10 120 python -c "$CHILD")"
    timeout -k 10 300 python -u bench.py --workload compress --no-cpu-baseline > gpurun_out/r06_rg_c_$v$run.json 2> gpurun_out/r06_rg_c_$v$run.err || { tail -20 gpurun_out/r06_rg_c_$v$run.err; exit 1; }
    python3 - gpurun_out/r06_rg_c_$v$run.json $v$run <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "compress", d["value"], "prove_only", d["prove_only"]["value"], flush=True)
PY
  done
done
unset ZKM_LIB
