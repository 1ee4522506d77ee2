# k_long_prep skipped for fused-stats sets (k_stats_long first on aux again): full GPU suite, then
# cfg4 x8 shards / cfg4 / cfg3 A/B vs libgkarray_hip_base.so (a53b900 + docs).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05E}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
for rep in 1 2; do
  for lib in libgkarray_hip.so libgkarray_hip_base.so; do
    export GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib
    timeout -k 10 300 python bench.py --workload cfg4 --virtual-shards 8 --no-cpu --steps 3 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg4 k8 $lib" | tee -a gpurun_out/${TAG}_ab.txt
    timeout -k 10 300 python bench.py --workload cfg4 --no-cpu --steps 3 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg4 k1 $lib" | tee -a gpurun_out/${TAG}_ab.txt
    timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg3 $lib" | tee -a gpurun_out/${TAG}_ab.txt
    timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 3 --streams 125000 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg3 S=125k $lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
