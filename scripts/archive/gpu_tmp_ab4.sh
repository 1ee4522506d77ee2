cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r03M
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|Timeout" gpurun_out/${TAG}_pytest.log | head; tail -30 gpurun_out/${TAG}_pytest.log | cut -c1-200; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for lib in libgkarray_hip.so libgkarray_hip_eagerhc.so libgkarray_hip.so libgkarray_hip_eagerhc.so; do
  GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python bench.py --workload cfg4 --virtual-shards 8 --no-cpu --steps 3 > gpurun_out/${TAG}_k8.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/${TAG}_k8.log; exit 1; }
  tail -1 gpurun_out/${TAG}_k8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg4 k8 $lib %.1f G ms/step %.2f' % (d['value']/1e9, d['ms_per_step']))" | tee -a gpurun_out/${TAG}_ab.txt
  GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 3 > gpurun_out/${TAG}_c5.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/${TAG}_c5.log; exit 1; }
  tail -1 gpurun_out/${TAG}_c5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg5 $lib ms/step %.2f launch_ms %.2f' % (d['ms_per_step'], d['roofline']['launch_ms']))" | tee -a gpurun_out/${TAG}_ab.txt
done
GK_HC_TRACE=1 timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 2 --warmup 1 > gpurun_out/${TAG}_hctrace.log 2>&1 || exit $?
grep "host chains" gpurun_out/${TAG}_hctrace.log | tail -2
