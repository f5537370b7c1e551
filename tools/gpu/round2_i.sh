# device trace generation: parity of the zkm_*_events_to_trace kernels against the host trace builders,
# the pinned/zero-copy host-trace test, then the tracegen bench and its kernel trace
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2i
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 600 python -u -m pytest tests/test_tracegen.py -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -20
timeout -k 10 300 python bench.py --workload tracegen --log-n 22 --steps 20 --warmup 2 > $O/bench_tracegen.json 2> $O/bench_tracegen.err || { tail -20 $O/bench_tracegen.err; exit 1; }
cat $O/bench_tracegen.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --workload tracegen --log-n 22 --steps 10 --warmup 1 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
echo done
