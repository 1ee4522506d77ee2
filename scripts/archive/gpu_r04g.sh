# Round-4: the half-wave kernel (GK_HALF=1) parity + A/B, the full GPU suite
# on the product library, and a rocprofv3 kernel trace of cfg5 with
# k_ingest_wg on.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
L=sketches-py_amd/gkarray_amd
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-36s %7.2f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
GK_HALF=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dist.py tests/test_gpu_configs.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_half_tests.log 2>&1
rc=$?
log "GK_HALF=1 tests rc=$rc: $(tail -1 gpurun_out/${TAG}_half_tests.log)"
grep -E "^E  " gpurun_out/${TAG}_half_tests.log | head -12 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
for rep in 1 2; do
  bline product || exit 1
  bline half4 GK_HALF=1 || exit 1
  bline half5 GK_HALF=1 GK_LIB_PATH=$L/libgkarray_hip_h5.so || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_full.log 2>&1
rc=$?
log "product full -m gpu rc=$rc: $(tail -1 gpurun_out/${TAG}_full.log)"
grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_full.log | head -20 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
D=gpurun_out/prof_${TAG}_cfg5
mkdir -p $D
GK_WG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > $D/bench.log 2>&1
log "cfg5 profile rc=$?: $(tail -1 $D/bench.log | cut -c1-200)"
