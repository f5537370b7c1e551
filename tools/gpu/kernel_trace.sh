# kernel-trace summary of the default bench workload: bash gpurun_prof.sh <tag>
set -e
TAG=${1:-cur}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 3 --warmup 1 --log-n 22 --no-cpu-baseline > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/kstats_$TAG.csv \;
tail -1 $R/gpurun_out/prof_$TAG.log | cut -c1-300
