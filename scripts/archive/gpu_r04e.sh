# Round-4 iteration: full GPU tests of chosen files on the product library,
# a quick parity check of each variant build, a cfg3 bench A/B of the builds
# that pass, then cfg5 with k_ingest_wg on / off.
# Usage: gpu_r04e.sh TAG "FULL_TESTS" lib1 lib2 ...   (lib1 = the product library)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; FULL=$2; shift 2
QUICK="tests/test_dist.py::test_gpu_fold_of_virtual_row_shards tests/test_gpu_parity.py::test_golden_streams tests/test_gpu_parity.py::test_golden_merges"
timeout -k 10 600 python -u -m pytest $FULL -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_full.log 2>&1
rc=$?
echo "product full tests rc=$rc: $(tail -1 gpurun_out/${TAG}_full.log)" | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then echo "abort (rc $rc)"; exit 1; fi
ok=""
for lib in "$@"; do
  GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python -u -m pytest $QUICK -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_q_${lib}.log 2>&1
  rc=$?
  echo "$lib quick rc=$rc: $(tail -1 gpurun_out/${TAG}_q_${lib}.log)" | tee -a gpurun_out/${TAG}_ab.txt
  if [ $rc -eq 0 ]; then ok="$ok $lib"; fi
  if [ $rc -gt 1 ]; then echo "abort (rc $rc)"; exit 1; fi
done
for rep in 1 2; do
  for lib in libgkarray_hip_r03.so $ok; do
    GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED: $lib"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-32s %7.2f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
# the two-streams-per-wave experiment (GK_HALF=1): parity first, then the bench
GK_HALF=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dist.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_half_tests.log 2>&1
rc=$?
echo "GK_HALF=1 tests rc=$rc: $(tail -1 gpurun_out/${TAG}_half_tests.log)" | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then echo "abort (rc $rc)"; exit 1; fi
if [ $rc -eq 0 ]; then
  for rep in 1 2; do
    for lib in libgkarray_hip.so libgkarray_hip_h5.so; do
      GK_HALF=1 GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED half: $lib"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('HALF %-27s %7.2f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$lib" | tee -a gpurun_out/${TAG}_ab.txt
    done
  done
fi
for wg in 1 0; do
  GK_WG=$wg timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 5 --warmup 2 > gpurun_out/${TAG}_cfg5_wg$wg.json 2> gpurun_out/${TAG}_cfg5_wg$wg.err || { echo "cfg5 FAILED wg=$wg"; tail -20 gpurun_out/${TAG}_cfg5_wg$wg.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_cfg5_wg$wg.json').read().strip().splitlines()[-1]); print('cfg5 GK_WG=%s  %7.3f Gv/s  ms/step %.2f' % (sys.argv[1], d['value']/1e9, d['ms_per_step']))" "$wg" | tee -a gpurun_out/${TAG}_ab.txt
done
