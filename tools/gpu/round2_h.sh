# zero-copy experiment: the transpose kernel reads pinned host traces over PCIe (ZKM_ZERO_COPY=1) vs
# DMA copies; parity of the host path first
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2h
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
ZKM_ZERO_COPY=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_prover.py tests/test_c_abi_host.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests_zc.log 2>&1 || { tail -30 $O/tests_zc.log; exit 1; }
tail -3 $O/tests_zc.log
for zc in 0 1; do
  ZKM_ZERO_COPY=$zc timeout -k 10 600 python bench.py --no-pmc --no-cpu-baseline > $O/bench_zc$zc.json 2> $O/bench_zc$zc.err || { tail -20 $O/bench_zc$zc.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_zc$zc.json').read().strip().splitlines()[-1]); print('zc=$zc pipelined', d['ms_per_shard'], 'per_call', d['host_per_call']['ms_per_shard'], 'resident', d['resident']['ms_per_shard'], 'serial', d['serial_ms_per_shard'])"
done
echo done
