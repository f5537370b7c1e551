# H2D FIFO stream + same-height LDE batching: GPU suite, bench fib (default), bench core, kernel trace of core.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2b
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=20 > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -25 $O/tests.log
timeout -k 10 600 python bench.py --no-cpu-baseline --no-pmc > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
timeout -k 10 600 python bench.py --workload core --no-cpu-baseline --no-pmc > $O/bench_core.json 2> $O/bench_core.err || { tail -30 $O/bench_core.err; exit 1; }
cut -c1-400 $O/bench_core.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_core -o run -- python3 $R/bench.py --workload core --inflight 1 --no-cpu-baseline --no-pmc > $O/trace_core.log 2>&1 || { tail -20 $O/trace_core.log; exit 1; }
echo done
