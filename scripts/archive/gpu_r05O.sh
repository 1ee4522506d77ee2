# EXPERIMENT: balanced small-class grid (GK_SMALL_BALANCE=1): cfg4 1 GPU (10^4 long streams), cfg3, S=125k.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05O}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for rep in 1 2; do
  for b in 0 1; do
    export GK_SMALL_BALANCE=$b
    timeout -k 10 300 python bench.py --workload cfg4 --no-cpu --steps 3 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg4 k1 balance=$b" | tee -a gpurun_out/${TAG}_ab.txt
    timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 --streams 125000 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg3 S=125k balance=$b" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
