# cfg5 (k_ingest_wg) iteration: wg / presort / spec-chain / cfg5 parity on the FIRST build, then the cfg5 bench
# interleaved over every listed build (REPS rounds, 10 steps).  Usage: gpu_r6_cfg5.sh TAG lib1 [lib2 ...]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
L=sketches-py_amd/gkarray_amd
if [ -z "$NOTEST" ]; then
  GK_LIB_PATH=$L/$1 timeout -k 10 600 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_presort.py tests/test_gpu_spec_chain.py \
    "tests/test_gpu_configs.py::test_cfg5_zipf_lengths_vs_oracle" tests/test_gpu_limits.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/${TAG}_pytest.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
fi
for rep in $(seq 1 ${REPS:-3}); do
  for lib in "$@"; do
    GK_LIB_PATH=$L/$lib timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 \
      > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED: $lib"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('cfg5 %-28s %7.2f Gv/s  ms/step %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step']))" "$lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
