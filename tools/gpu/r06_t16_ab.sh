# Round 6 A/B: the 2^23 LDE with tile-major intermediates (k_ntt_s10 1024 x 16 tiles + k_lde_fused13s<16>; B = in-tree)
# against row-major ones (A = zkmips_amd/libzkm_hip_a.so): 2^23 parity tests first, then the LDE microbench
# alternated in fresh processes.  gpurun_out/r06_t16_*
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prover.py -x -q -m gpu -k "23 or lde" --timeout 300 --timeout-method thread > gpurun_out/r06_t16_tests.log 2>&1 || { tail -30 gpurun_out/r06_t16_tests.log; exit 1; }
tail -2 gpurun_out/r06_t16_tests.log
CHILD="import sys; sys.path.insert(0, '$R'); from zkmips_amd._lib import Device; d = Device(0); print(' '.join('%.4f' % d.bench_lde(1 << L, W, 10) for L, W in [(23, 64), (23, 44), (22, 64)]))"
echo "LDE ms: 2^23x64 2^23x44 2^22x64"
for run in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export ZKM_LIB=$R/zkmips_amd/libzkm_hip_a.so; else unset ZKM_LIB; fi
    echo "$v$run $(timeout -k 10 120 python -c "$CHILD")"
  done
done
unset ZKM_LIB
