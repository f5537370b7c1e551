# MemoryLocal + Global chips, headline-size parity tests, pipelined bench, core bench.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2c
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread --durations=15 > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -20 $O/tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 600 python bench.py --workload core --no-cpu-baseline --no-pmc > $O/bench_core.json 2> $O/bench_core.err || { tail -30 $O/bench_core.err; exit 1; }
cut -c1-300 $O/bench_core.json
echo done
