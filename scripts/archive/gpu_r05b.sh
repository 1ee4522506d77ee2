# Round-5 iteration: the wg / host-chain / parity tests touched by the
# presort and join fixes, then the cfg5 and cfg3 bench lines.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05b}
timeout -k 10 600 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_hostchains.py tests/test_gpu_presort.py \
  tests/test_gpu_spec_chain.py tests/test_gpu_configs.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
for rep in 1 2; do
timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}_bench_cfg5.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_cfg5.log | cut -c1-200
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/${TAG}_bench_cfg3.log 2>&1 || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_bench_cfg3.log').read().strip().splitlines()[-1]); print('cfg3 %.2f Gv/s ms/step %.3f launch %.3f frac %.4f' % (d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))"
done
