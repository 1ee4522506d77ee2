# Round-4: k_ingest_wg section profile (presorted vs unsorted batches), cfg5
# A/B of wave priority for k_stats_long, host-chain tests with default env.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
L=sketches-py_amd/gkarray_amd
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; local wl=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu --workload $wl --steps 5 --warmup 2 > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-40s %7.3f Gv/s  ms/step %.3f  launch_ms %.3f  stats_ms %s' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline'].get('stats_kernel_ms')))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
for ps in 0 1; do
  GK_WG_PRESORT=$ps GK_HOST_CHAINS=0 timeout -k 10 200 python tools/prof_sections.py --workload wg > gpurun_out/${TAG}_sections_ps$ps.txt 2>&1 || { log "prof failed"; tail -5 gpurun_out/${TAG}_sections_ps$ps.txt; exit 1; }
  log "== wg sections, GK_WG_PRESORT=$ps"; cat gpurun_out/${TAG}_sections_ps$ps.txt | tee -a gpurun_out/${TAG}_ab.txt
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_hostchains.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
log "hostchain tests rc=$rc: $(tail -1 gpurun_out/${TAG}_tests.log)"
if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
for rep in 1 2; do
  bline wg_presort_prio cfg5 GK_HOST_CHAINS=0 GK_WG=1 GK_WG_PRESORT=1 || exit 1
  bline wg_presort_noprio cfg5 GK_HOST_CHAINS=0 GK_WG=1 GK_WG_PRESORT=1 GK_SL_PRIO=0 || exit 1
  bline wg_nopresort cfg5 GK_HOST_CHAINS=0 GK_WG=1 || exit 1
done
