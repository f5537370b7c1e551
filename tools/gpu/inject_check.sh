set -e
O=$GRAFT_REPO_ROOT/gpurun_out/inject
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_mips_core.py tests/test_memory_global.py tests/test_mips_alu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "commit or identical or full_size" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 600 python bench.py --workload core --no-cpu-baseline --no-pmc > $O/bench_core.json 2> $O/bench_core.err || { tail -30 $O/bench_core.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_core.json'));print('core', d['ms_per_shard'], d['resident']['ms_per_shard'], d['serial_ms_per_shard'], {k:v['ms_per_shard'] for k,v in d['stages_ms_per_shard'].items() if k in ('merkle_nodes','merkle_leaves','lde')})"
