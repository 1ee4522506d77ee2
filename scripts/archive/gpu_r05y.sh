# EXPERIMENT: the cost of the per-call block on the previous call (may_defer) -- cfg3 proxies with and without it.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05y}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for nb in 0 1; do
  if [ $nb = 1 ]; then export GK_EXP_NOBLOCK=1; fi
  timeout -k 10 300 python tools/host_enqueue.py 125000 1000000 2>&1 | grep -v amdgpu.ids | sed "s/^/noblock=$nb /" | tee -a gpurun_out/${TAG}_host.txt
  for S in 1000000 125000; do
    timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 --streams $S > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg3 S=$S noblock=$nb" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
