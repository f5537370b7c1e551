# Round 6: kernel trace of the 64-leaf compress tree (--workload compress), stats under gpurun_out/r06_ctrace*
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_ctrace -o run -- python3 $R/bench.py --workload compress --no-cpu-baseline > $R/gpurun_out/r06_ctrace.log 2>&1 || { tail -20 $R/gpurun_out/r06_ctrace.log; exit 1; }
find $R/gpurun_out/r06_ctrace -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r06_ctrace_stats.csv \;
tail -1 $R/gpurun_out/r06_ctrace.log | cut -c1-300
