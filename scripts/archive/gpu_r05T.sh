# cfg5: the capacity-class launch beside k_ingest_wg on fewer waves (GK_CLS_GRID_PCT) -- does a lighter
# chip (power, memory traffic) shorten the workgroup flush chain?  bench lines only, 2 reps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05T}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for rep in 1 2; do
  for pct in 100 60 35 20; do
    GK_CLS_GRID_PCT=$pct timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 GRID_PCT=$pct" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
