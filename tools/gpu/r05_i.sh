#!/bin/bash
# round 5, call i: kernel trace of serial single-shard proofs (one slot in flight): the FRI commit-phase
# timeline and the opening launches of one proof, with nothing overlapping them
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/r05i_trace -o fib -- python3 $R/bench.py --inflight 1 --steps 2 --warmup 1 --no-cpu-baseline --no-maxshape --no-compress --no-tendermint --no-sizes --no-pmc > $O/r05i.json 2> $O/r05i.err || { tail -20 $O/r05i.err; exit 1; }
find $O/r05i_trace -name "*kernel_trace.csv" -exec cp {} $O/r05i_ktrace.csv \;
cd $R
python3 tools/timeline.py $O/r05i_ktrace.csv -1 > $O/r05i_fri_timeline.txt
tail -12 $O/r05i_fri_timeline.txt
