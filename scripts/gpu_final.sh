# Round-end evidence: scripts/gpu_round.sh (tests, smoke, bench lines, cfg4
# allocation trace, cfg3 trace + PMC), then the default bench line again with
# the freshly stamped PMC traffic, the 2-rank rehearsal of the N-GPU bench on
# this one GPU, and the all-cores CPU-baseline leg.  Usage: gpu_final.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final}
bash scripts/gpu_round.sh $TAG || exit $?
cp gpurun_out/prof_$TAG/pmc_traffic.json profiles/pmc_traffic.json || exit 1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_final.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_final.log | cut -c1-400
GK_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_rehearse_n2.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_rehearse_n2.log | cut -c1-300
timeout -k 10 400 python bench.py --cpu-all-cores --steps 3 > gpurun_out/${TAG}_bench_allcores.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_allcores.log | cut -c1-200
