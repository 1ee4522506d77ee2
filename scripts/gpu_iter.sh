# One build->measure iteration on the GPU box: the -m gpu suite on the
# product library, then an A/B of the default bench (cfg3) against other
# builds.  Usage: gpu_iter.sh TAG [libname ...]   (lib names in gkarray_amd/)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
for rep in 1 2; do
  for lib in libgkarray_hip.so "$@"; do
    GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED: $lib"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-32s %7.2f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
