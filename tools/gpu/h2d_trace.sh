# kernel + memory-copy timeline of the host-trace bench (3 in flight, plain async copies)
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/h2d_trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
ZKM_H2D_FIFO=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/t -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-pmc --inflight 3 --steps 3 --warmup 1 > $O/log 2>&1 || { tail -20 $O/log; exit 1; }
tail -c 300 $O/log
