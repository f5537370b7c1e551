# default bench line (as the driver runs it) + a 2-rank sha2 execution rehearsal on one GPU (config 4 path)
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
ZKM_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --workload sha2 --sha-blocks 2048 --gpus 2 --steps 2 --warmup 1 > gpurun_out/r02_bench_sha2_rehearse2.json 2> gpurun_out/r02_bench_sha2_rehearse2.err || { tail -20 gpurun_out/r02_bench_sha2_rehearse2.err; exit 1; }
cut -c1-400 gpurun_out/r02_bench_sha2_rehearse2.json
timeout -k 10 600 python -u bench.py > gpurun_out/r02_bench_default.json 2> gpurun_out/r02_bench_default.err || { tail -20 gpurun_out/r02_bench_default.err; exit 1; }
cut -c1-600 gpurun_out/r02_bench_default.json
