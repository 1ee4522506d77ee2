cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r03Q
timeout -k 10 300 python -u -m pytest tests/test_gpu_presort.py tests/test_gpu_configs.py::test_cfg5_zipf_lengths_vs_oracle tests/test_gpu_hostchains.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/${TAG}_pytest1.log 2>&1 || { echo "pytest1 failed"; grep -E "FAILED|Error|Timeout" gpurun_out/${TAG}_pytest1.log | head; tail -30 gpurun_out/${TAG}_pytest1.log | cut -c1-200; exit 1; }
tail -1 gpurun_out/${TAG}_pytest1.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 3 > gpurun_out/${TAG}_c5.log 2>&1 || { echo "cfg5 failed"; tail -5 gpurun_out/${TAG}_c5.log; exit 1; }
  tail -1 gpurun_out/${TAG}_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('wave presort ms/step %.2f launch_ms %.2f stats_ms %.2f' % (d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['stats_kernel_ms']))" | tee -a gpurun_out/${TAG}_c5.txt
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|Timeout" gpurun_out/${TAG}_pytest.log | head; tail -30 gpurun_out/${TAG}_pytest.log | cut -c1-200; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_c5trace -o run -- python3 bench.py --workload cfg5 --no-cpu --steps 2 --warmup 1 > gpurun_out/${TAG}_c5trace.log 2>&1 || exit $?
