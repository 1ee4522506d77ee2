# Stats-drain A/B: parity subset on the product build, then cfg3 and the
# 125k proxy over (library, environment) pairs, then timeline builds.
# Usage: gpu_r6_drain.sh TAG "lib1 ENV=a" "lib2" ...   (REPS; TL="lib ..."; NOPAR=1)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
L=sketches-py_amd/gkarray_amd
if [ -z "$NOPAR" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pq.log 2>&1 \
    || { echo "PARITY FAILED"; grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pq.log | head; exit 1; }
  echo "parity: $(tail -1 gpurun_out/${TAG}_pq.log)"
fi
CFGS=("$@")
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in "${CFGS[@]}"; do
    read -r lib envs <<< "$cfg"
    env GK_LIB_PATH=$L/$lib $envs timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 \
      > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED: $cfg"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-40s %7.2f Gv/s  ms/step %.4f  launch_ms %.4f  frac %.4f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$cfg" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in "${CFGS[@]}"; do
    read -r lib envs <<< "$cfg"
    env GK_LIB_PATH=$L/$lib $envs timeout -k 10 200 python bench.py --no-cpu --steps 50 --warmup 3 --proxy 8 \
      > gpurun_out/${TAG}_px.tmp 2>&1 || { echo "FAILED proxy: $cfg"; tail -20 gpurun_out/${TAG}_px.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_px.tmp').read().strip().splitlines()[-1]); print('proxy8 %-33s %7.2f Gv/s  ms/step %.4f  launch_ms %.4f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms']))" "$cfg" | tee -a gpurun_out/${TAG}_px.txt
  done
done
for t in $TL; do
  read -r lib envs <<< "${t//,/ }"
  env GK_LIB_PATH=$L/$lib $envs timeout -k 10 300 python3 tools/launch_timeline.py ${TL_S:-1000000} > gpurun_out/${TAG}_tl_${t//[ ,=]/_}.txt 2>&1 || { echo "timeline failed $t"; tail gpurun_out/${TAG}_tl.txt; exit 1; }
  echo "== $t"; head -12 gpurun_out/${TAG}_tl_${t//[ ,=]/_}.txt
done
