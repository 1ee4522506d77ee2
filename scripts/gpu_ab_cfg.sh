# A/B of library builds on one workload (default bench flags otherwise).
# Usage: gpu_ab_cfg.sh TAG WORKLOAD STEPS lib1 lib2 ...   (lib names in gkarray_amd/)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; W=$2; K=$3; shift 3
for rep in 1 2; do
  for lib in "$@"; do
    GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python bench.py --workload $W --no-cpu --steps $K --warmup 2 > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED: $lib"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-6s %-28s %7.2f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[2], sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$lib" "$W" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
