# recursion GPU tests + tracegen bench (incl. Poseidon2WideDeg3) + a 2-rank compress-tree rehearsal on one GPU
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_recursion.py tests/test_tracegen.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02_gpu_tests_rtg.log 2>&1 || { tail -30 gpurun_out/r02_gpu_tests_rtg.log; exit 1; }
tail -2 gpurun_out/r02_gpu_tests_rtg.log
timeout -k 10 300 python -u bench.py --workload tracegen --steps 5 --warmup 1 > gpurun_out/r02_bench_tracegen.json 2> gpurun_out/r02_bench_tracegen.err || { tail -20 gpurun_out/r02_bench_tracegen.err; exit 1; }
ZKM_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --workload compress --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r02_bench_compress_rehearse2.json 2> gpurun_out/r02_bench_compress_rehearse2.err || { tail -20 gpurun_out/r02_bench_compress_rehearse2.err; exit 1; }
cut -c1-300 gpurun_out/r02_bench_compress_rehearse2.json
