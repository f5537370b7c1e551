# host-trace throughput vs in-flight depth, with and without the FIFO H2D stream
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/h2d_sweep
mkdir -p $O
for f in 1 0; do for k in 3 5; do
  ZKM_H2D_FIFO=$f timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --inflight $k --steps 4 > $O/b_${f}_${k}.json 2> $O/b_${f}_${k}.err || { tail -20 $O/b_${f}_${k}.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_${f}_${k}.json'));print('fifo=$f inflight=$k', d['ms_per_shard'], d['resident']['ms_per_shard'])"
done; done
