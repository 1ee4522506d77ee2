# Round-4: promoted streams re-run by k_ingest_wg: full suite, A/B on cfg3 and
# the strong-split proxies, cfg3 trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r04x
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 5 $BARGS > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-32s %8.3f Gv/s  ms/step %.4f  launch_ms %.4f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms']))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_full.log 2>&1
rc=$?
log "full -m gpu rc=$rc: $(tail -1 gpurun_out/${TAG}_full.log)"
grep -E "^E  |^FAILED|^ERROR" gpurun_out/${TAG}_full.log | head -20 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -ne 0 ]; then log "abort (rc $rc)"; exit 1; fi
for rep in 1 2; do
  for S in 1000000 125000; do
    BARGS="--streams $S" bline "S=$S rerun_wg" || exit 1
    BARGS="--streams $S" bline "S=$S rerun_1wave" GK_RERUN_WG=0 || exit 1
  done
done
D=gpurun_out/prof_${TAG}_cfg3
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 > $D/bench.log 2>&1
log "cfg3 profile rc=$?"
