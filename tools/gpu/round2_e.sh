# syscall/SHA precompile shards GPU == oracle, then the full GPU suite (core machine now carries the SHA
# chips; their JIT kernels come from the in-tree code-object cache), then smoke
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2e
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
ls $R/zkmips_amd/jit_cache | wc -l > $O/jit_cache_files.txt
timeout -k 10 600 python -u -m pytest tests/test_syscall.py -x -v -m gpu --timeout 500 --timeout-method thread > $O/syscall.log 2>&1 || { tail -40 $O/syscall.log; exit 1; }
tail -3 $O/syscall.log
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread --durations=10 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -14 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log
