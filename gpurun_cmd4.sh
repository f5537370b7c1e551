set -e
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof4 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --log-n 22 --no-cpu-baseline > $R/gpurun_out/prof4.log 2>&1 || { tail -20 $R/gpurun_out/prof4.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --log-n 22 --no-cpu-baseline > $R/gpurun_out/pmc_fetch.log 2>&1 || { tail -20 $R/gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --log-n 22 --no-cpu-baseline > $R/gpurun_out/pmc_write.log 2>&1 || { tail -20 $R/gpurun_out/pmc_write.log; exit 1; }
find $R/gpurun_out/prof4 $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write -type f | head -20
