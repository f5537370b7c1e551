# SQ stall counters over one bench step: bash gpurun_pmc_sq.sh <tag>
set -e
TAG=${1:-sq}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/pmc_$TAG -o run -- python3 $R/bench.py --steps 1 --warmup 0 --log-n 22 --no-cpu-baseline > $R/gpurun_out/pmc_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_$TAG.log; exit 1; }
find $R/gpurun_out/pmc_$TAG -name "*counter_collection.csv" | head -3
