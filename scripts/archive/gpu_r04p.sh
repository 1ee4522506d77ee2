# Round-4: k_ingest_wg workgroup size A/B (4 / 8 / 16 waves) on cfg5 + wg tests
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
L=sketches-py_amd/gkarray_amd
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; local wl=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu --workload $wl --steps 5 --warmup 2 > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-40s %7.3f Gv/s  ms/step %.3f  launch_ms %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms']))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
for v in w16 w4; do
  GK_LIB_PATH=$L/libgkarray_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wg.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests_$v.log 2>&1
  rc=$?
  log "$v wg tests rc=$rc: $(tail -1 gpurun_out/${TAG}_tests_$v.log)"
  if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
done
for rep in 1 2; do
  bline wg8 cfg5 || exit 1
  bline wg16 cfg5 GK_LIB_PATH=$L/libgkarray_hip_w16.so || exit 1
  bline wg4 cfg5 GK_LIB_PATH=$L/libgkarray_hip_w4.so || exit 1
done
