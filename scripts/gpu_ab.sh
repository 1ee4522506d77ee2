# A/B of library builds on the default bench (cfg3) and cfg2.
# Usage: gpu_ab.sh TAG "ENV1=.. ENV2=.." "libname1 libname2 ..."   (lib names in sketches-py_amd/gkarray_amd)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
for cfg in "$@"; do
  for rep in 1 2; do
    env $cfg timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED: $cfg"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-60s %7.2f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$cfg" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
