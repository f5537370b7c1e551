# compress-tree bench line + kernel-trace summary of single compress proofs
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 400 python3 -u $R/bench.py --workload compress --steps 3 --warmup 1 > $R/gpurun_out/r02_bench_compress.json 2> $R/gpurun_out/r02_bench_compress.err || { tail -20 $R/gpurun_out/r02_bench_compress.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_compress -o run -- python3 $R/bench.py --workload compress --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline > $R/gpurun_out/prof_compress.log 2>&1 || { tail -20 $R/gpurun_out/prof_compress.log; exit 1; }
find $R/gpurun_out/prof_compress -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/kstats_compress.csv \;
cat $R/gpurun_out/r02_bench_compress.json | cut -c1-600
