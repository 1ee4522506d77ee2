# k_ingest_wg launched ahead of the chain walks and the presort (GK_WG_EARLY=1, its workgroups wait on the
# device for k_long_prep's word) vs behind them (=0): GPU parity (wg / presort / configs / spec / host
# chains), cfg5 A/B, and the workgroups' start times (timeline build).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05AG}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
timeout -k 10 700 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_presort.py tests/test_gpu_configs.py tests/test_gpu_spec_chain.py tests/test_gpu_hostchains.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
for rep in 1 2; do
  for e in 0 1; do
    GK_WG_EARLY=$e timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 EARLY=$e" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
TL_WARM=3 timeout -k 10 300 python3 tools/launch_timeline.py wg:cfg5 > gpurun_out/${TAG}_wg_clock.txt 2>&1 || exit $?
head -20 gpurun_out/${TAG}_wg_clock.txt
