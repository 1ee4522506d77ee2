cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for K in 8 1; do
  timeout -k 10 400 python bench.py --workload cfg4 --virtual-shards $K --no-cpu --steps 2 --warmup 1 > gpurun_out/cfg4_k$K.log 2>&1 || { tail -20 gpurun_out/cfg4_k$K.log; exit 1; }
  tail -1 gpurun_out/cfg4_k$K.log | cut -c1-700
done
