# Stats-role A/B over libraries (GK_LIB_PATH) and GK_FUSED_STATS values
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-fab}
for lib in ${LIBS:-libgkarray_hip.so}; do
  for f in ${FS_LIST:-3}; do
    for w in cfg3 cfg2; do
      GK_LIB_PATH=$PWD/sketches-py_amd/gkarray_amd/$lib GK_FUSED_STATS=$f timeout -k 10 300 python bench.py --workload $w --no-cpu --steps 5 > gpurun_out/${TAG}_${lib}_${w}_f$f.log 2>&1 || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], sys.argv[4], 'Gv/s=%.2f ms/step=%.3f launch_ms=%.3f' % (d['value']/1e9, d['ms_per_step'], r['launch_ms']))" gpurun_out/${TAG}_${lib}_${w}_f$f.log $lib $w f$f | tee -a gpurun_out/${TAG}_ab.txt
    done
  done
done
