# MIPS core shard: bench line + kernel-trace summary (single shard in flight)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u bench.py --workload core --steps 3 --warmup 1 --no-cpu-baseline --no-pmc > gpurun_out/r02_bench_core_latest.json 2> gpurun_out/r02_bench_core_latest.err || { tail -20 gpurun_out/r02_bench_core_latest.err; exit 1; }
cut -c1-300 gpurun_out/r02_bench_core_latest.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_core -o run -- python3 $R/bench.py --workload core --steps 2 --warmup 1 --inflight 1 --no-cpu-baseline --no-pmc > $R/gpurun_out/prof_core.log 2>&1 || { tail -20 $R/gpurun_out/prof_core.log; exit 1; }
find $R/gpurun_out/prof_core -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/kstats_core.csv \;
