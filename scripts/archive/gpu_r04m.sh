# Round-4: register presort (k_presort_reg), presort only for k_ingest_wg's
# streams, one-wave launch beside the presort: full suite, cfg5 A/B, trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; local wl=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu --workload $wl --steps 5 --warmup 2 > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-40s %7.3f Gv/s  ms/step %.3f  launch_ms %.3f  stats_ms %s' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline'].get('stats_kernel_ms')))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_full.log 2>&1
rc=$?
log "full -m gpu rc=$rc: $(tail -1 gpurun_out/${TAG}_full.log)"
grep -E "^E  |^FAILED|^ERROR" gpurun_out/${TAG}_full.log | head -20 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -ne 0 ]; then log "abort (rc $rc)"; exit 1; fi
for rep in 1 2; do
  bline cfg5_default_regpresort cfg5 || exit 1
  bline cfg5_ldspresort cfg5 GK_PRESORT_REG=0 || exit 1
  bline cfg5_nopresort cfg5 GK_WG_PRESORT=0 || exit 1
done
bline cfg3 cfg3 || exit 1
D=gpurun_out/prof_${TAG}_cfg5
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > $D/bench.log 2>&1
log "cfg5 profile rc=$?"
