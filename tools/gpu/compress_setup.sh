# compress bench line incl. the per-program setup time
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python3 -u bench.py --workload compress --steps 3 --warmup 1 > gpurun_out/r02_bench_compress_setup.json 2> gpurun_out/r02_bench_compress_setup.err || { tail -20 gpurun_out/r02_bench_compress_setup.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r02_bench_compress_setup.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_proof'], d['serial_ms_per_proof'], d['setup_ms_per_program'])"
