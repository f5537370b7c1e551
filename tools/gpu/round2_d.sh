# full GPU suite (2^22 random core shard restored), default bench line with PMC, and kernel trace of the default bench
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2d
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 1100 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread --durations=12 > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -16 $O/tests.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-pmc > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace1 -o run -- python3 $R/bench.py --inflight 1 --steps 4 --no-cpu-baseline --no-pmc > $O/trace1.log 2>&1 || { tail -20 $O/trace1.log; exit 1; }
echo done
