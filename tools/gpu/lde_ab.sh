# A/B of LDE kernel variants: bash tools/gpu/lde_ab.sh <ENVVAR> <values...>
# LDE parity tests under each variant, then the 2^22 x 67 microbench (kernel trace per variant).
set -e
VAR=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/ab
cat > /tmp/ldeb.py <<PY
import sys; sys.path.insert(0,'$R')
from zkmips_amd._lib import Device
d=Device(0)
for lg,w in [(22,67),(22,44),(20,67)]:
    print('lde 2^%d x %d: %.3f ms'%(lg,w,d.bench_lde(1<<lg,w,int(sys.argv[1]))))
PY
for v in "$@"; do
  export $VAR=$v
  timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -x -q -k lde > $R/gpurun_out/ab/t_$v.log 2>&1 || { echo "variant $v FAILED"; tail -30 $R/gpurun_out/ab/t_$v.log; exit 1; }
  echo "$VAR=$v: $(tail -1 $R/gpurun_out/ab/t_$v.log)"
  timeout -k 10 120 python3 /tmp/ldeb.py 10
done
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  export $VAR=$v
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab/kt_$v -o run -- python3 /tmp/ldeb.py 3 > $R/gpurun_out/ab/kt_$v.log 2>&1 || { tail $R/gpurun_out/ab/kt_$v.log; exit 1; }
  echo "== $VAR=$v"; python3 -c "import csv,sys; [print(r[\"Name\"][:50].ljust(50), r[\"Calls\"], round(float(r[\"AverageNs\"])/1e3,1)) for r in csv.DictReader(open(sys.argv[1]))]" $(find $R/gpurun_out/ab/kt_$v -name "*kernel_stats.csv")
done
