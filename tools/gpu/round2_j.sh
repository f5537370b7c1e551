# LDS evidence for the Poseidon2 (Merkle) and NTT kernels: SQ LDS counters over one 2^22 FibCpu proof
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2j
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -E "SQ_INSTS_LDS|SQ_LDS_BANK_CONFLICT|SQ_LDS_IDX_ACTIVE|SQ_INSTS_VALU\b|SQ_WAVES\b|SQ_ACTIVE_INST_LDS|SQ_LDS_ADDR_CONFLICT" $O/counters.txt | head -20 || true
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/lds -o run -- python3 $R/bench.py --pmc-child --workload fib --log-n 22 > $O/lds.log 2>&1 || { tail -20 $O/lds.log; exit 1; }
find $O/lds -name "*counter_collection.csv" | head -2
echo done
