# EXPERIMENT: k_ingest_wg launched first (GK_WG_FIRST) and/or alone on its CUs (GK_WG_EXCL): cfg5 A/B + wg parity.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05J}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
GK_WG_FIRST=1 GK_WG_EXCL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head; exit 1; }
echo "tests ok with GK_WG_FIRST=1 GK_WG_EXCL=1"; tail -1 gpurun_out/${TAG}_pytest.log
for rep in 1 2; do
  for cfg in "0 0" "1 0" "1 1" "0 1"; do
    set -- $cfg
    GK_WG_FIRST=$1 GK_WG_EXCL=$2 timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 FIRST=$1 EXCL=$2" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
GK_WG_FIRST=1 GK_WG_EXCL=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_trace -o run -- \
  python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > gpurun_out/${TAG}_trace.log 2>&1 || exit $?
f=$(find gpurun_out/${TAG}_trace -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py "$f" | head -20
