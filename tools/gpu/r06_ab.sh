# Round 6 A/B of two library builds by kernel trace: ZKM_LIB=zkmips_amd/libzkm_hip_a.so (A) vs the in-tree
# libzkm_hip.so (B), alternated twice, default FibCpu 2^22 main leg only; per-kernel stats under gpurun_out/r06_<tag>_{A,B}{1,2}
set -e
TAG=${1:-ab}
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for run in 1 2; do
  for v in A B; do
    if [ $v = A ]; then export ZKM_LIB=$R/zkmips_amd/libzkm_hip_a.so; else unset ZKM_LIB; fi
    D=$R/gpurun_out/r06_${TAG}_$v$run
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 $R/bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-maxshape --no-compress --no-tendermint --no-sizes --no-pmc > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
    find $D -name "*kernel_stats.csv" -exec cp {} $D.csv \;
    tail -1 $D.log | cut -c1-200
  done
done
unset ZKM_LIB
