# Round profile for profiles/: the default bench line, the kernel-trace summary of the same command,
# the same for one shard in flight (--inflight 1), and HBM PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs, kernel dispatch only).
# Run on the GPU box from the repo root:  bash tools/gpu/profile_round.sh
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace1 -o run -- python3 $R/bench.py --inflight 1 --no-cpu-baseline > $O/trace1.log 2>&1 || { tail -20 $O/trace1.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/fetch.log 2>&1 || { tail -20 $O/fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/write.log 2>&1 || { tail -20 $O/write.log; exit 1; }
echo profiled
