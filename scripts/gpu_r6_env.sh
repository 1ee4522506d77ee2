# A/B over (library, environment) pairs on the default bench (cfg3), interleaved.
# Usage: gpu_r6_env.sh TAG "lib1 ENV=a ENV2=b" "lib2" ...   (REPS, BENCH_ARGS; TL="lib ..." timeline builds)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
L=sketches-py_amd/gkarray_amd
CFGS=("$@")
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in "${CFGS[@]}"; do
    read -r lib envs <<< "$cfg"
    env GK_LIB_PATH=$L/$lib $envs timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 ${BENCH_ARGS} \
      > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED: $cfg"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-44s %7.2f Gv/s  ms/step %.4f  launch_ms %.4f  frac %.4f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$cfg" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
for lib in $TL; do
  GK_LIB_PATH=$L/$lib timeout -k 10 300 python3 tools/launch_timeline.py 1000000 > gpurun_out/${TAG}_tl_${lib}.txt 2>&1 || { echo "timeline failed $lib"; tail gpurun_out/${TAG}_tl_${lib}.txt; exit 1; }
  echo "== $lib"; cat gpurun_out/${TAG}_tl_${lib}.txt
done
