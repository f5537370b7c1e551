# LDE microbench (2^22 x 67): kernel-trace stats + two SQ counter passes.  bash tools/gpu/lde_prof.sh <tag>
set -e
TAG=${1:-x}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ldep_$TAG
mkdir -p $O
cat > /tmp/ldeb.py <<PY
import sys; sys.path.insert(0,'$R')
from zkmips_amd._lib import Device
d=Device(0)
print('lde 2^22 x 67: %.3f ms'%d.bench_lde(1<<22,67,int(sys.argv[1])))
PY
timeout -k 10 120 python3 /tmp/ldeb.py 10 > $O/plain.log 2>&1 || { tail $O/plain.log; exit 1; }
cat $O/plain.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 /tmp/ldeb.py 5 > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/sq1 -o run -- python3 /tmp/ldeb.py 2 > $O/sq1.log 2>&1 || { tail $O/sq1.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS --output-format csv -d $O/sq2 -o run -- python3 /tmp/ldeb.py 2 > $O/sq2.log 2>&1 || { tail $O/sq2.log; exit 1; }
cd $R
python3 tools/sq_summary.py $(find $O/sq1 $O/sq2 -name "*counter_collection.csv") > $O/sq.txt
cat $O/sq.txt
python3 tools/kstats.py $(find $O/kt -name "*kernel_stats.csv") 6
