# Round-6 build->measure iteration: the -m gpu suite on the FIRST listed
# build (GK_LIB_PATH), then the default bench (cfg3) interleaved over every
# listed build (REPS rounds), then one SQ pass (VALU/SALU/LDS counts) per build.
# Usage: gpu_r6.sh TAG lib1 [lib2 ...]   (lib names in sketches-py_amd/gkarray_amd/)
#        NOTEST=1 skips the suite; REPS (default 3); SQ=0 skips the counters.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
L=sketches-py_amd/gkarray_amd
if [ -z "$NOTEST" ]; then
  GK_LIB_PATH=$L/$1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -2 gpurun_out/${TAG}_pytest.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
fi
for rep in $(seq 1 ${REPS:-3}); do
  for lib in "$@"; do
    GK_LIB_PATH=$L/$lib timeout -k 10 200 python bench.py --no-cpu --steps 20 --warmup 3 ${BENCH_ARGS} \
      > gpurun_out/${TAG}_ab.tmp 2>&1 || { echo "FAILED: $lib"; tail -20 gpurun_out/${TAG}_ab.tmp; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-28s %7.2f Gv/s  ms/step %.4f  launch_ms %.4f  frac %.4f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
[ "${SQ:-1}" = "0" ] && exit 0
for lib in "$@"; do
  n=${lib#libgkarray_hip}; n=${n%.so}; n=${n#_}; [ -z "$n" ] && n=prod
  GK_LIB_PATH=$L/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
    --kernel-include-regex k_ingest_small --output-format csv -d gpurun_out/${TAG}_${n}_p1 -o run -- \
    python3 bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/${TAG}_${n}_p1.log 2>&1 || { echo "SQ pass failed: $lib"; tail -5 gpurun_out/${TAG}_${n}_p1.log; exit 1; }
  echo "$n: $(python3 tools/sq_summary.py ${TAG}_${n} | grep -E 'VALU/flush|SALU/flush|LDS/flush' | tr -s ' ' | tr '\n' ';')"
done
