set -e
O=$GRAFT_REPO_ROOT/gpurun_out/dma_probe
mkdir -p $O
for p in 0 1; do
ZKM_BENCH_DMA_PROBE=$p timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --steps 10 > $O/b_$p.json 2> $O/b_$p.err || { tail -20 $O/b_$p.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_$p.json'));print('probe=$p', d['ms_per_shard'], d['host_per_call']['ms_per_shard'], d['resident']['ms_per_shard'])"
done
