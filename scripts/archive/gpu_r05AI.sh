# the two-phase presort (r05V) on top of the early workgroup launch: GPU parity at the default ka and at
# ka=100, then cfg5 A/B against the committed library (libgkarray_hip_base.so) over GK_WG_PSA.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05AI}
D=sketches-py_amd/gkarray_amd
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_presort.py tests/test_gpu_configs.py tests/test_gpu_spec_chain.py tests/test_gpu_hostchains.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
GK_WG_PSA=100 timeout -k 10 400 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_presort.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_ka100.log 2>&1
rc=$?; echo "pytest ka=100 rc=$rc"; tail -1 gpurun_out/${TAG}_pytest_ka100.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest_ka100.log | head -20; exit 1; fi
for rep in 1 2; do
  GK_LIB_PATH=$D/libgkarray_hip_base.so timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
  line gpurun_out/${TAG}.tmp "cfg5 committed" | tee -a gpurun_out/${TAG}_ab.txt
  for ka in 0 1500 2300 3200; do
    GK_WG_PSA=$ka timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 two-phase PSA=$ka" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
