# Round-4: 8-ary gap search in k_ingest_wg (A/B vs binary), wg tests,
# section profile; SQ counters of k_ingest_small (product, GD16 variant) and
# of the half-wave kernel (GK_HALF=1) for DESIGN 6.1.
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
timeout -k 10 400 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_configs.py tests/test_gpu_presort.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
log "tests rc=$rc: $(tail -1 gpurun_out/${TAG}_tests.log)"
grep -E "^E  |^FAILED" gpurun_out/${TAG}_tests.log | head -12 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -ne 0 ]; then log "abort (rc $rc)"; exit 1; fi
timeout -k 10 200 python tools/prof_sections.py --workload wg > gpurun_out/${TAG}_sections.txt 2>&1 || { log "prof failed"; exit 1; }
log "== wg sections (presorted, 8-ary)"; grep -v amdgpu.ids gpurun_out/${TAG}_sections.txt | tee -a gpurun_out/${TAG}_ab.txt
for rep in 1 2; do
  bline cfg5_search8 cfg5 || exit 1
  bline cfg5_search2 cfg5 GK_LIB_PATH=$L/libgkarray_hip_s2.so || exit 1
done
bash scripts/pmc_sq.sh ${TAG}_sq_prod > gpurun_out/${TAG}_sq_prod.log 2>&1 || { log "sq prod failed"; exit 1; }
GK_LIB_PATH=$L/libgkarray_hip_gd.so bash scripts/pmc_sq.sh ${TAG}_sq_gd > gpurun_out/${TAG}_sq_gd.log 2>&1 || { log "sq gd failed"; exit 1; }
GK_HALF=1 KRX=k_ingest_half bash scripts/pmc_sq.sh ${TAG}_sq_half > gpurun_out/${TAG}_sq_half.log 2>&1 || { log "sq half failed"; exit 1; }
python3 tools/sq_summary.py ${TAG}_sq_prod ${TAG}_sq_gd | tee -a gpurun_out/${TAG}_ab.txt
KRX=k_ingest_half python3 tools/sq_summary.py ${TAG}_sq_half | tee -a gpurun_out/${TAG}_ab.txt
