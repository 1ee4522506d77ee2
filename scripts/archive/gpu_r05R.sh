# per-batch presort readiness (readiness words, batch-major presort order) vs the whole-presort flag
# (GK_WG_BFLAGS=0): GPU parity on the wg / presort / configs / spec / host-chain tests, then cfg5 A/B + trace.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05R}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_presort.py tests/test_gpu_configs.py tests/test_gpu_spec_chain.py tests/test_gpu_hostchains.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
for rep in 1 2; do
  for bf in 1 0; do
    GK_WG_BFLAGS=$bf timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 BFLAGS=$bf" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
  python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
f=$(find gpurun_out/${TAG}_trace -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" | head -12
