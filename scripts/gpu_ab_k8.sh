# A/B of library builds on cfg4 with 8 virtual row shards.  Usage: gpu_ab_k8.sh TAG lib1 lib2 ...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python bench.py --workload cfg4 --virtual-shards 8 --no-cpu --steps 3 --warmup 1 > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED: $lib"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('cfg4k8 %-28s %7.2f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
