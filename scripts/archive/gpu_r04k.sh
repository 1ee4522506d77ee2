# Round-4: k_ingest_wg with register-resident carry walk + fused member rank:
# parity, section profile, cfg5 A/B presort vs none.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; local wl=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu --workload $wl --steps 5 --warmup 2 > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-40s %7.3f Gv/s  ms/step %.3f  launch_ms %.3f  stats_ms %s' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline'].get('stats_kernel_ms')))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
GK_WG=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_configs.py tests/test_gpu_presort.py tests/test_gpu_spec_chain.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
log "tests rc=$rc: $(tail -1 gpurun_out/${TAG}_tests.log)"
grep -E "^E  |^FAILED" gpurun_out/${TAG}_tests.log | head -12 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -ne 0 ]; then log "abort (rc $rc)"; exit 1; fi
for ps in 0 1; do
  GK_WG_PRESORT=$ps GK_HOST_CHAINS=0 timeout -k 10 200 python tools/prof_sections.py --workload wg > gpurun_out/${TAG}_sections_ps$ps.txt 2>&1 || { log "prof failed"; tail -5 gpurun_out/${TAG}_sections_ps$ps.txt; exit 1; }
  log "== wg sections, GK_WG_PRESORT=$ps"; grep -v amdgpu.ids gpurun_out/${TAG}_sections_ps$ps.txt | tee -a gpurun_out/${TAG}_ab.txt
done
for rep in 1 2; do
  bline wg_presort cfg5 GK_HOST_CHAINS=0 GK_WG=1 GK_WG_PRESORT=1 || exit 1
  bline wg_nopresort cfg5 GK_HOST_CHAINS=0 GK_WG=1 || exit 1
done
