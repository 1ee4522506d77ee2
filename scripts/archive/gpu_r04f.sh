# Round-4 iteration (one box, many questions): full GPU tests of the product
# library (and a bisect of variants only if they fail), a cfg3 A/B, the
# half-wave experiment, cfg5 with k_ingest_wg on / off, strong-split proxies.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
L=sketches-py_amd/gkarray_amd
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {  # name env... : one bench line summary
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-36s %7.2f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_full.log 2>&1
rc=$?
log "product full -m gpu rc=$rc: $(tail -1 gpurun_out/${TAG}_full.log)"
grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_full.log | head -20 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
QUICK="tests/test_dist.py::test_gpu_fold_of_virtual_row_shards tests/test_gpu_parity.py::test_golden_streams tests/test_gpu_parity.py::test_golden_merges tests/test_gpu_parity.py::test_random_batches_vs_oracle"
ok=""
for lib in libgkarray_hip_gd.so libgkarray_hip_dpp.so libgkarray_hip_tp.so libgkarray_hip_zs.so libgkarray_hip_all.so; do
  GK_LIB_PATH=$L/$lib timeout -k 10 300 python -u -m pytest $QUICK -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_q_${lib}.log 2>&1
  r=$?
  log "$lib quick rc=$r: $(tail -1 gpurun_out/${TAG}_q_${lib}.log)"
  if [ $r -gt 1 ] && [ $r -ne 4 ]; then log "abort (rc $r)"; exit 1; fi
  if [ $r -eq 0 ]; then ok="$ok $lib"; fi
done
for rep in 1 2; do
  bline r03 GK_LIB_PATH=$L/libgkarray_hip_r03.so || exit 1
  bline product GK_LIB_PATH=$L/libgkarray_hip.so || exit 1
  for lib in $ok; do bline $lib GK_LIB_PATH=$L/$lib || exit 1; done
  bline o5-lds-5waves GK_LIB_PATH=$L/libgkarray_hip_o5.so || exit 1
  bline product-FS8 GK_FUSED_STATS=8 || exit 1
done
GK_HALF=1 GK_LIB_PATH=$L/libgkarray_hip_all.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dist.py tests/test_gpu_configs.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_half_tests.log 2>&1
rc=$?
log "GK_HALF=1 tests rc=$rc: $(tail -1 gpurun_out/${TAG}_half_tests.log)"
grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_half_tests.log | head -10 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
for rep in 1 2; do
  bline half4 GK_HALF=1 GK_LIB_PATH=$L/libgkarray_hip_all.so || exit 1
  bline half5 GK_HALF=1 GK_LIB_PATH=$L/libgkarray_hip_allh5.so || exit 1
done
for wg in 1 0; do
  GK_WG=$wg timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 5 --warmup 2 > gpurun_out/${TAG}_cfg5_wg$wg.json 2> gpurun_out/${TAG}_cfg5_wg$wg.err || { log "cfg5 FAILED wg=$wg"; tail -20 gpurun_out/${TAG}_cfg5_wg$wg.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_cfg5_wg$wg.json').read().strip().splitlines()[-1]); print('cfg5 GK_WG=%s  %7.3f Gv/s  ms/step %.2f' % (sys.argv[1], d['value']/1e9, d['ms_per_step']))" "$wg" | tee -a gpurun_out/${TAG}_ab.txt
done
for S in 500000 250000 125000; do
  timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 --streams $S > gpurun_out/${TAG}_proxy_$S.json 2>&1 || { log "proxy FAILED $S"; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_proxy_$S.json').read().strip().splitlines()[-1]); print('proxy S=%s  %7.2f Gv/s  ms/step %.3f  launch_ms %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms']))" "$S" | tee -a gpurun_out/${TAG}_ab.txt
done
