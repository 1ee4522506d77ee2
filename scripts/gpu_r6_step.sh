# Per-step overhead A/B: the -m gpu suite on the product build (NOTEST=1
# skips), the 125k-stream proxy and cfg3 over the listed builds (interleaved,
# REPS), then a kernel trace of the proxy step on each listed build.
# Usage: gpu_r6_step.sh TAG lib1 [lib2 ...]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
L=sketches-py_amd/gkarray_amd
if [ -z "$NOTEST" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/${TAG}_pytest.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
fi
for rep in $(seq 1 ${REPS:-3}); do
  for lib in "$@"; do
    GK_LIB_PATH=$L/$lib timeout -k 10 200 python bench.py --no-cpu --steps 50 --warmup 3 --proxy 8 \
      > gpurun_out/${TAG}_px.tmp 2>&1 || { echo "FAILED proxy: $lib"; tail -20 gpurun_out/${TAG}_px.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_px.tmp').read().strip().splitlines()[-1]); print('proxy8 %-26s %7.2f Gv/s  ms/step %.4f  launch_ms %.4f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms']))" "$lib" | tee -a gpurun_out/${TAG}_px.txt
    GK_LIB_PATH=$L/$lib timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 \
      > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED: $lib"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('cfg3   %-26s %7.2f Gv/s  ms/step %.4f  launch_ms %.4f  frac %.4f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
for lib in "$@"; do
  n=${lib%.so}; n=${n#libgkarray_hip}; n=${n#_}; [ -z "$n" ] && n=prod
  GK_LIB_PATH=$L/$lib timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_${n}_kt -o run -- \
    python3 bench.py --no-cpu --proxy 8 --steps 30 --warmup 3 > gpurun_out/${TAG}_${n}_kt.log 2>&1 || { echo "trace failed $lib"; tail -5 gpurun_out/${TAG}_${n}_kt.log; exit 1; }
  f=$(find gpurun_out/${TAG}_${n}_kt -name "*kernel_trace.csv" | head -1)
  python3 tools/step_timeline.py $f > gpurun_out/${TAG}_${n}_step.txt || exit 1
  echo "== $lib"; tail -16 gpurun_out/${TAG}_${n}_step.txt
done
