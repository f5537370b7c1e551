# the default bench line as the driver runs it + a kernel-trace summary of the same workload
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u bench.py > gpurun_out/r02_bench_final.json 2> gpurun_out/r02_bench_final.err || { tail -20 gpurun_out/r02_bench_final.err; exit 1; }
cut -c1-300 gpurun_out/r02_bench_final.json
bash tools/gpu/kernel_trace.sh r02final
