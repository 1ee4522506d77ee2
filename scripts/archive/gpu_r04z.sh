# Round-4: the strong-split N-rank path rehearsed on one GPU (both ranks share
# the card: a path check, not a scaling number)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
GK_BENCH_REHEARSE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r04z_rehearse_n2.json 2> gpurun_out/r04z_rehearse_n2.err
echo "rc=$?" >> gpurun_out/r04z_rehearse_n2.err
tail -1 gpurun_out/r04z_rehearse_n2.json | cut -c1-600
