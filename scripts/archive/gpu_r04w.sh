# Round-4: the stats role at the strong split's per-rank sizes: proxies
# S = 125k / 250k / 500k with GK_FUSED_STATS 7 (default) / 8 / 4 / 0
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r04w
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 5 $BARGS > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-32s %8.3f Gv/s  ms/step %.4f  launch_ms %.4f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms']))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
for S in 125000 250000 500000; do
  for fs in 7 8 4 0; do
    BARGS="--streams $S" bline "S=$S FS=$fs" GK_FUSED_STATS=$fs || exit 1
  done
done
