cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r03t
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 3 > gpurun_out/${TAG}_bench_cfg5.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench_cfg5.log | cut -c1-200
tail -1 gpurun_out/${TAG}_bench_cfg5.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline'])"
for v in rk1 rk2; do
  GK_LIB_PATH=sketches-py_amd/gkarray_amd/libgkarray_hip_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_$v.log 2>&1 || { echo "pytest $v failed"; tail -30 gpurun_out/${TAG}_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest_$v.log
done
bash scripts/gpu_ab.sh $TAG "GK_LIB_PATH=sketches-py_amd/gkarray_amd/libgkarray_hip.so" "GK_LIB_PATH=sketches-py_amd/gkarray_amd/libgkarray_hip_rk1.so" "GK_LIB_PATH=sketches-py_amd/gkarray_amd/libgkarray_hip_rk2.so" "GK_LIB_PATH=sketches-py_amd/gkarray_amd/libgkarray_hip.so" || exit 1
bash scripts/lds_attrib.sh $TAG libgkarray_hip.so libgkarray_hip_rk1.so libgkarray_hip_rk2.so
