# wg iteration: parity (wg, presort, configs), cfg5 A/B vs the committed library, per-wave profile.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05p}
timeout -k 10 600 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_presort.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
for rep in 1 2; do
  for lib in libgkarray_hip.so libgkarray_hip_emit.so libgkarray_hip_merged.so libgkarray_hip_head.so; do
    GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 $lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
GK_WG_CONC=0 timeout -k 10 300 python tools/prof_sections.py --workload wg --per-wave > gpurun_out/${TAG}_wg_perwave_seq.txt 2>&1 || exit $?
head -16 gpurun_out/${TAG}_wg_perwave_seq.txt
