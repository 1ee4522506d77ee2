# two-phase presort beside k_ingest_wg (batches 1..ka-1 of its streams first, published apart): GPU parity at the
# default ka and at ka=100 (both phases inside the test streams), then cfg5 A/B over GK_WG_PSA + trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05V}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_presort.py tests/test_gpu_configs.py tests/test_gpu_spec_chain.py tests/test_gpu_hostchains.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
GK_WG_PSA=100 timeout -k 10 400 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_presort.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_ka100.log 2>&1
rc=$?; echo "pytest ka=100 rc=$rc"; tail -1 gpurun_out/${TAG}_pytest_ka100.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest_ka100.log | head -20; exit 1; fi
for rep in 1 2; do
  for ka in 0 1500 2300 3200; do
    GK_WG_PSA=$ka timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 PSA=$ka" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
  python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
f=$(find gpurun_out/${TAG}_trace -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" > gpurun_out/${TAG}_timeline.txt; head -14 gpurun_out/${TAG}_timeline.txt
