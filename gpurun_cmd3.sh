set -e
mkdir -p gpurun_out
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --log-n 22 > gpurun_out/bench3.json 2> gpurun_out/bench3.err || { tail -30 gpurun_out/bench3.err; exit 1; }
cat gpurun_out/bench3.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --log-n 22 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof3.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof3.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof3 -name "*stats*" | head
