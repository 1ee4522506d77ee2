cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
true
for rep in 1 2; do for lib in libgkarray_hip.so libgkarray_hip_w7.so libgkarray_hip_w8.so libgkarray_hip_r02.so; do
  GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/r03l_ab.tmp 2>&1 || { echo "FAILED: $lib"; tail -5 gpurun_out/r03l_ab.tmp; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r03l_ab.tmp').read().strip().splitlines()[-1]); print('%-28s %7.2f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$lib" | tee -a gpurun_out/r03l_ab.txt
done; done
