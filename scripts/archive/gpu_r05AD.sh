# the occupancy query cached (once per kernel instead of per launch) vs the base library: host enqueue per
# step (tools/host_enqueue.py) and cfg3 bench at 125k / 1M streams; 2 reps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05AD}
D=sketches-py_amd/gkarray_amd
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for v in hip_base hip; do
  GK_LIB_PATH=$D/lib${v/hip/gkarray_hip}.so timeout -k 10 300 python3 tools/host_enqueue.py 125000 2>&1 | grep "S=" | sed "s/^/$v /" | tee -a gpurun_out/${TAG}_ab.txt
done
for rep in 1 2; do
  for S in 125000 1000000; do
    for v in hip_base hip; do
      GK_LIB_PATH=$D/lib${v/hip/gkarray_hip}.so timeout -k 10 300 python bench.py --streams $S --no-cpu --steps 20 --warmup 3 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
      line gpurun_out/${TAG}.tmp "S=$S $v" | tee -a gpurun_out/${TAG}_ab.txt
    done
  done
done
