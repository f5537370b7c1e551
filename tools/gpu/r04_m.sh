#!/bin/bash
# round 4, call m (final evidence): the default bench line, then a rocprofv3 kernel-trace summary of the headline
# command (timed regions + profiled region; in-run counter passes and secondary legs off so the profiler sees
# the prover only) whose k_hash_leaves average must agree with the line's roofline.avg_ms
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 900 python3 -u bench.py --steps 10 --warmup 2 > $O/r04m_bench.log 2>&1 || { tail -30 $O/r04m_bench.log; exit 1; }
tail -1 $O/r04m_bench.log | cut -c1-300
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/r04m_prof -o run --output-format csv -- python3 -u bench.py --steps 5 --warmup 1 --no-pmc --no-sizes --no-maxshape --no-compress --no-tendermint --no-cpu-baseline > $O/r04m_prof_bench.log 2>&1 || { tail -30 $O/r04m_prof_bench.log; exit 1; }
tail -1 $O/r04m_prof_bench.log | cut -c1-200
find $O/r04m_prof -name "*kernel_stats.csv" | head -3
