# round-2 final: full GPU suite (oracle now AVX-512), default bench line (PMC + CPU baseline at 2^22),
# kernel trace of the default bench, and the sha2-execution (config 3) bench
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2g
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread --durations=10 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -14 $O/tests.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
timeout -k 10 600 python bench.py --workload sha2 --steps 3 > $O/bench_sha2.json 2> $O/bench_sha2.err || { tail -30 $O/bench_sha2.err; exit 1; }
cut -c1-600 $O/bench_sha2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --no-cpu-baseline --no-pmc > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }

timeout -k 10 300 python3 $R/tools/gpu/dma_uncached.py > $O/dma_uncached.txt 2>&1 || { tail -20 $O/dma_uncached.txt; exit 1; }
cat $O/dma_uncached.txt
echo done
