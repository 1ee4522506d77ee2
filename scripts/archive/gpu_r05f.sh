# Pipelined workgroup gaps: wg / cfg5 parity, cfg5 bench A/B, wg section profile.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05f}
timeout -k 10 600 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_presort.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}_cfg5.log 2>&1 || exit $?
  line gpurun_out/${TAG}_cfg5.log cfg5 | tee -a gpurun_out/${TAG}_ab.txt
done
GK_WG_PRESORT=1 timeout -k 10 300 python tools/prof_sections.py --workload wg > gpurun_out/${TAG}_wg_sections.txt 2>&1 || exit $?
cat gpurun_out/${TAG}_wg_sections.txt
