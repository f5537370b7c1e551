set -e
O=$GRAFT_REPO_ROOT/gpurun_out/sdma_probe
mkdir -p $O
for sd in 1 0; do for k in 2 4; do
HSA_ENABLE_SDMA=$sd timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --steps 10 --inflight $k > $O/b_${sd}_$k.json 2> $O/b_${sd}_$k.err || { tail -20 $O/b_${sd}_$k.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_${sd}_$k.json'));print('sdma=$sd k=$k', d['ms_per_shard'], d['host_per_call']['ms_per_shard'], d['resident']['ms_per_shard'])"
done; done
