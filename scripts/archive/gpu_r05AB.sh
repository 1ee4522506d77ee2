# the host's wait on the previous call (may_defer): polling the event (GK_SPIN_WAIT=1) vs hipEventSynchronize
# (=0); cfg3 at 1M and 125k streams, host-timed enqueue loop + bench; 2 reps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05AB}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for rep in 1 2; do
  for S in 125000 1000000; do
    for sp in 0 1; do
      GK_SPIN_WAIT=$sp timeout -k 10 300 python bench.py --streams $S --no-cpu --steps 20 --warmup 3 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
      line gpurun_out/${TAG}.tmp "S=$S spin=$sp" | tee -a gpurun_out/${TAG}_ab.txt
    done
  done
done
