# compress tree throughput vs proofs in flight
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/cinf
cd $R
for k in 2 3 4 6; do
  timeout -k 10 300 python3 -u bench.py --workload compress --steps 3 --warmup 1 --inflight $k --no-cpu-baseline > gpurun_out/cinf/b_$k.json 2> gpurun_out/cinf/b_$k.err || { tail -20 gpurun_out/cinf/b_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/cinf/b_$k.json').read().strip().splitlines()[-1]); print('inflight $k', d['value'], d['ms_per_step'], d['ms_per_proof'])"
done
