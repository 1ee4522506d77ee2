# cfg5 A/B of workgroup sizes (4 / 8 / 16 waves per long stream), wg parity on each.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05l}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for lib in libgkarray_hip_w16.so libgkarray_hip_w4.so; do
  GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_wg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_$lib.log 2>&1 || { echo "FAILED tests $lib"; grep -E "FAILED|Error" gpurun_out/${TAG}_pytest_$lib.log | head; exit 1; }
done
echo "wg tests ok on variants"
for rep in 1 2; do
  for lib in libgkarray_hip.so libgkarray_hip_head.so libgkarray_hip_w16.so libgkarray_hip_w4.so; do
    GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 $lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_cfg5trace -o run -- \
  python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > gpurun_out/${TAG}_cfg5trace.log 2>&1 || exit $?
echo traced
# cfg5 strong-split proxies: every rank's balanced_assignment share alone
for N in 2 4 8; do
  R=0
  while [ $R -lt $N ]; do
    timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 5 --warmup 1 --proxy $N --proxy-rank $R > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 proxy N=$N rank=$R" | tee -a gpurun_out/${TAG}_proxy.txt
    R=$((R+1))
  done
done
