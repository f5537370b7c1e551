# Round 2, first GPU pass: full -m gpu suite (local_only fix), the bench line (host-trace headline,
# in-run PMC traffic) and a kernel-trace summary of the default bench command.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2a
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-pmc > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
echo done
