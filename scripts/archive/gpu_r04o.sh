# Round-4: every-flush register sort in k_ingest_small (GK_SORTALL variant):
# parity + cfg3 A/B; cfg5 default bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
L=sketches-py_amd/gkarray_amd
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; local wl=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu --workload $wl --steps 10 --warmup 3 > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-40s %7.3f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
GK_LIB_PATH=$L/libgkarray_hip_sa.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
log "sortall tests rc=$rc: $(tail -1 gpurun_out/${TAG}_tests.log)"
grep -E "^E  |^FAILED" gpurun_out/${TAG}_tests.log | head -12 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
for rep in 1 2; do
  bline product cfg3 || exit 1
  bline sortall cfg3 GK_LIB_PATH=$L/libgkarray_hip_sa.so || exit 1
done
bline cfg5 cfg5 || exit 1
