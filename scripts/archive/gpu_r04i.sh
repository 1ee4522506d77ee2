# Round-4: speculative k_stats_long + k_ingest_wg without presort: parity,
# then cfg5 A/B and a kernel trace.
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
GK_WG=1 GK_HOST_CHAINS=0 timeout -k 10 500 python -u -m pytest tests/test_gpu_spec_chain.py tests/test_gpu_wg.py tests/test_gpu_hostchains.py tests/test_gpu_configs.py tests/test_gpu_presort.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
log "tests rc=$rc: $(tail -1 gpurun_out/${TAG}_tests.log)"
grep -E "^E  |^FAILED" gpurun_out/${TAG}_tests.log | head -12 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
for rep in 1 2; do
  bline wg_nopresort cfg5 GK_HOST_CHAINS=0 GK_WG=1 || exit 1
  bline wg_presort cfg5 GK_HOST_CHAINS=0 GK_WG=1 GK_WG_PRESORT=1 || exit 1
  bline wg_nopresort_noprio cfg5 GK_HOST_CHAINS=0 GK_WG=1 GK_SL_PRIO=0 || exit 1
  bline wg_nopresort_w32 cfg5 GK_HOST_CHAINS=0 GK_WG=1 GK_LIB_PATH=$L/libgkarray_hip_w32.so || exit 1
  bline wg_nopresort_hc cfg5 GK_WG=1 || exit 1
done
bline cfg3_product cfg3 || exit 1
bline cfg4_wg_hc0 cfg4 GK_HOST_CHAINS=0 GK_WG=1 || exit 1
bline cfg4_product cfg4 || exit 1
D=gpurun_out/prof_${TAG}_cfg5
mkdir -p $D
GK_HOST_CHAINS=0 GK_WG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > $D/bench.log 2>&1
log "cfg5 profile rc=$?"
