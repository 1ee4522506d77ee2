# workgroup size A/B with the round-5 flush: 8 (product) / 12 / 16 waves; wg parity on each variant.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05F}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for lib in libgkarray_hip_w16.so libgkarray_hip_w12.so; do
  GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_wg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_$lib.log 2>&1 || { echo "FAILED tests $lib"; grep -E "FAILED|Error" gpurun_out/${TAG}_pytest_$lib.log | head; exit 1; }
done
echo "wg tests ok on variants"
for lib in libgkarray_hip.so libgkarray_hip_w16.so libgkarray_hip_w12.so; do
  GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 120 python tools/wg_alone.py 1 10000000 3 2>&1 | grep "per flush" | sed "s/^/$lib /"
done
for rep in 1 2; do
  for lib in libgkarray_hip.so libgkarray_hip_w16.so libgkarray_hip_w12.so; do
    GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 $lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
