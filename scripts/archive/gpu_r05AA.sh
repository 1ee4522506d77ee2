# bench with the warm-up extended to >= 0.3 s (GPU clock ramp) vs the old W-steps-only warm-up
# (GK_BENCH_MIN_WARM_S=0): cfg3 at 1M and the strong-split proxy sizes, cfg5; 2 reps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05AA}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f warm %s' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['warmup_run']['steps']))" "$@"; }
for rep in 1 2; do
  for S in 1000000 500000 250000 125000; do
    for mw in 0 0.3; do
      GK_BENCH_MIN_WARM_S=$mw timeout -k 10 300 python bench.py --streams $S --no-cpu --steps 20 --warmup 3 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
      line gpurun_out/${TAG}.tmp "S=$S min_warm=$mw" | tee -a gpurun_out/${TAG}_ab.txt
    done
  done
  for mw in 0 0.3; do
    GK_BENCH_MIN_WARM_S=$mw timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 min_warm=$mw" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
