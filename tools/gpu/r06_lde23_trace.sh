# Round 6: kernel trace of the 2^23 x 64 LDE microbench (zkm_bench_lde), stats under gpurun_out/r06_lde23*
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r06_lde23 -o run -- python3 -c "import sys; sys.path.insert(0, '$R'); from zkmips_amd._lib import Device; d = Device(0); print('%.4f ms' % d.bench_lde(1 << 23, 64, 10)); print('%.4f ms' % d.bench_lde(1 << 22, 64, 10))" > $R/gpurun_out/r06_lde23.log 2>&1 || { tail -20 $R/gpurun_out/r06_lde23.log; exit 1; }
find $R/gpurun_out/r06_lde23 -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/r06_lde23_stats.csv \;
grep ' ms' $R/gpurun_out/r06_lde23.log
