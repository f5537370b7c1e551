#!/bin/bash
# round 4, call a: the default bench line (value = resident), H2D attribution kernel traces
# (pipelined vs resident), and SQ/TA counter passes over the LDE microbench (strided-pass stall).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
timeout -k 10 700 python3 -u bench.py --steps 10 --warmup 2 --no-compress > $O/r04a_bench.log 2>&1 || { tail -30 $O/r04a_bench.log; exit 1; }
tail -1 $O/r04a_bench.log | cut -c1-400
for mode in resident pipelined; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r04a_kt_$mode -o run -- \
    python3 tools/h2d_attrib.py $mode 6 > $O/r04a_kt_$mode.log 2>&1 || { tail -20 $O/r04a_kt_$mode.log; exit 1; }
  find $O/r04a_kt_$mode -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/r04a_kstats_$mode.csv
  tail -1 $O/r04a_kt_$mode.log
done
python3 tools/kdelta.py $O/r04a_kstats_resident.csv $O/r04a_kstats_pipelined.csv resident pipelined > $O/r04a_h2d_delta.txt
head -30 $O/r04a_h2d_delta.txt
cat > /tmp/ldeb.py <<PY
import sys; sys.path.insert(0, '$GRAFT_REPO_ROOT')
from zkmips_amd._lib import Device
d = Device(0)
print('lde %.2f ms' % d.bench_lde(1 << 22, 67, 3))
PY
cd /tmp
R=$GRAFT_REPO_ROOT/$O
timeout -k 10 120 rocprofv3 -L > $R/r04a_counters.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $R/r04a_pmc1 -o run -- python3 /tmp/ldeb.py > $R/r04a_pmc1.log 2>&1 || { tail -5 $R/r04a_pmc1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS --output-format csv -d $R/r04a_pmc2 -o run -- python3 /tmp/ldeb.py > $R/r04a_pmc2.log 2>&1 || { tail -5 $R/r04a_pmc2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $R/r04a_pmc3 -o run -- python3 /tmp/ldeb.py > $R/r04a_pmc3.log 2>&1 || { tail -5 $R/r04a_pmc3.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d $R/r04a_pmc4 -o run -- python3 /tmp/ldeb.py > $R/r04a_pmc4.log 2>&1 || { tail -5 $R/r04a_pmc4.log; exit 1; }
if grep -q 'TA_BUSY_avr' $R/r04a_counters.txt && grep -q 'TA_TA_BUSY' $R/r04a_counters.txt; then
  timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_BUFFER_READ_WAVEFRONTS_sum --output-format csv -d $R/r04a_pmc5 -o run -- python3 /tmp/ldeb.py > $R/r04a_pmc5.log 2>&1 || { tail -5 $R/r04a_pmc5.log; exit 1; }
fi
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_compress_tree.py -m gpu > $O/r04a_gpu_compress_test.log 2>&1 || { tail -30 $O/r04a_gpu_compress_test.log; exit 1; }
tail -3 $O/r04a_gpu_compress_test.log
timeout -k 10 500 python3 -u bench.py --workload compress --no-cpu-baseline > $O/r04a_compress.log 2>&1 || { tail -30 $O/r04a_compress.log; exit 1; }
tail -1 $O/r04a_compress.log | cut -c1-600
echo done
