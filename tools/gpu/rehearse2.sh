# 2-rank rehearsal of bench.py's N>1 flow on a 1-GPU box (ranks share the card, gloo collectives).
set -e
mkdir -p gpurun_out
ZKM_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err || { tail -30 gpurun_out/rehearse2.err; exit 1; }
cut -c1-400 gpurun_out/rehearse2.json
