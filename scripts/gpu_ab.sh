cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ab}
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then tail -60 gpurun_out/${TAG}_pytest.log | cut -c1-300; exit 1; fi
for rep in 1 2; do
for lib in libgkarray_hip.so libgkarray_hip_lb0.so; do
  GK_LIB_PATH=$GRAFT_REPO_ROOT/sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_$lib.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$lib', 'Gv/s=%.2f'%(d['value']/1e9), 'ms/step=%.2f'%d['ms_per_step'], 'ingest_ms=%.2f'%r['launch_ms'], 'stats_ms=%.2f'%r['stats_kernel_ms'], 'GB/s=%.0f'%r['achieved'])"
done
done
