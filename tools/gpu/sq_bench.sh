# Per-kernel SQ counters + kernel trace over one single-shard bench step: bash tools/gpu/sq_bench.sh <tag> [bench args]
set -e
TAG=${1:-sq}; shift || true
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/sqb_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 1 --warmup 1 --inflight 1 --profile-steps 1 --no-cpu-baseline "$@" > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/sq1 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --inflight 1 --profile-steps 1 --no-cpu-baseline "$@" > $O/sq1.log 2>&1 || { tail -20 $O/sq1.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $O/sq2 -o run -- python3 $R/bench.py --steps 1 --warmup 0 --inflight 1 --profile-steps 1 --no-cpu-baseline "$@" > $O/sq2.log 2>&1 || { tail -20 $O/sq2.log; exit 1; }
cd $R
python3 tools/sq_summary.py $(find $O/sq1 $O/sq2 -name "*counter_collection.csv") > $O/sq.txt
head -30 $O/sq.txt | cut -c1-230
