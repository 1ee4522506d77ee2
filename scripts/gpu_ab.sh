# A/B of library variants on the default bench workload:  bash scripts/gpu_ab.sh TAG lib1 lib2 ...
# (libs are file names under sketches-py_amd/gkarray_amd/, built with `make variant`)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ab}; shift
WL=${WL:-cfg3}
for rep in 1 2; do
for lib in "$@"; do
  GK_LIB_PATH=$GRAFT_REPO_ROOT/sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python bench.py --workload $WL --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_$lib.log 2>&1 || exit $?
  tail -1 gpurun_out/${TAG}_$lib.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$lib', 'Gv/s=%.2f'%(d['value']/1e9), 'ms/step=%.2f'%d['ms_per_step'], 'ingest_ms=%.2f'%r['launch_ms'], 'stats_ms=%.2f'%r['stats_kernel_ms'], 'GB/s=%.0f'%r['achieved'])"
done
done
