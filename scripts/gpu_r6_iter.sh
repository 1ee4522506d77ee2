# Round-6 iteration: gpu_r6.sh (suite on the first build, cfg3 A/B, SQ), then
# the 125k-stream strong-split proxy (one rank's share of 8) A/B, then the
# section profile of the profiling build.  Usage: gpu_r6_iter.sh TAG lib1 [lib2 ...]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
bash scripts/gpu_r6.sh "$@" || exit $?
shift
if [ -n "$PROXY" ]; then
  for rep in 1 2; do
    for lib in "$@"; do
      GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 200 python bench.py --no-cpu --steps 50 --warmup 3 --proxy 8 \
        > gpurun_out/${TAG}_px.tmp 2>&1 || { echo "FAILED proxy: $lib"; tail -20 gpurun_out/${TAG}_px.tmp; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_px.tmp').read().strip().splitlines()[-1]); print('proxy8 %-24s %7.2f Gv/s  ms/step %.4f  launch_ms %.4f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms']))" "$lib" | tee -a gpurun_out/${TAG}_px.txt
    done
  done
fi
if [ -n "$SECPROF" ]; then
  timeout -k 10 300 python3 tools/prof_sections.py --workload cfg3 > gpurun_out/${TAG}_sec_cfg3.txt 2>&1 || exit $?
  cat gpurun_out/${TAG}_sec_cfg3.txt
fi
