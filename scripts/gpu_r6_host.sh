# Round 6 item 2/3 evidence: kernel traces of the 125k-stream proxy step (product vs round-5 library),
# the per-step timeline, and the 2-rank rehearsal line (per-rank roofline fields).  Usage: gpu_r6_host.sh TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-host}
L=sketches-py_amd/gkarray_amd
for lib in libgkarray_hip.so libgkarray_hip_r5.so; do
  n=${lib%.so}; n=${n#libgkarray_hip}; n=${n#_}; [ -z "$n" ] && n=prod
  GK_LIB_PATH=$L/$lib timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_${n}_kt -o run -- \
    python3 bench.py --no-cpu --proxy 8 --steps 30 --warmup 3 > gpurun_out/${TAG}_${n}_kt.log 2>&1 || { echo "trace failed $lib"; tail -5 gpurun_out/${TAG}_${n}_kt.log; exit 1; }
  f=$(find gpurun_out/${TAG}_${n}_kt -name "*kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py $f > gpurun_out/${TAG}_${n}_step.txt || exit 1
  echo "== $lib"; tail -1 gpurun_out/${TAG}_${n}_kt.log | cut -c1-160; tail -30 gpurun_out/${TAG}_${n}_step.txt
done
GK_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_rehearse_n2.log 2>&1 || { tail -20 gpurun_out/${TAG}_rehearse_n2.log; exit 1; }
tail -1 gpurun_out/${TAG}_rehearse_n2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('n_gpus', d['n_gpus'], 'rank', r['rank'], 'launch_ms', r['launch_ms'], 'frac', r['frac']); [print(x) for x in r['per_rank']]"
