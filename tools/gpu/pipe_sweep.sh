# pipelined host-trace bench vs in-flight depth
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/pipe_sweep
mkdir -p $O
for k in 2 3 4; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --inflight $k --steps 4 > $O/b_$k.json 2> $O/b_$k.err || { tail -20 $O/b_$k.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$k.json'));print('inflight=$k', d['ms_per_shard'], d['host_per_call']['ms_per_shard'], d['resident']['ms_per_shard'], d['serial_ms_per_shard'])"
done
