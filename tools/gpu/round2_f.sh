# maximal-shape MIPS shard: byte parity at Cpu 2^18, full-size prove + verify; SysLinux shards; the
# maxshape bench line and its kernel trace
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2f
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 900 python -u -m pytest tests/test_shapes.py tests/test_syscall.py -x -v -m gpu --timeout 600 --timeout-method thread --durations=5 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -12 $O/tests.log
timeout -k 10 900 python bench.py --workload maxshape --steps 4 --no-cpu-baseline > $O/bench_maxshape.json 2> $O/bench_maxshape.err || { tail -30 $O/bench_maxshape.err; exit 1; }
cut -c1-400 $O/bench_maxshape.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --workload maxshape --steps 2 --inflight 1 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
echo done
