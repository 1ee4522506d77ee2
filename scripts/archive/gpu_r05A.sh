# wg LDS layout A/B: padded value slots + (g, d) pairs (libgkarray_hip.so) vs libgkarray_hip_base.so:
# wg/presort/spec parity, wg alone (S=1) time + LDS bank conflicts, cfg5 bench.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05A}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_wg.py tests/test_gpu_presort.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
for lib in libgkarray_hip.so libgkarray_hip_base.so; do
  export GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib
  timeout -k 10 120 python tools/wg_alone.py 1 10000000 3 2>&1 | grep "per flush" | sed "s/^/$lib /"
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex k_ingest_wg --output-format csv \
    -d gpurun_out/${TAG}_pmc_$lib -o run -- python3 tools/wg_alone.py 1 10000000 2 > gpurun_out/${TAG}_pmc_$lib.log 2>&1 || { echo "pmc failed"; tail -3 gpurun_out/${TAG}_pmc_$lib.log; exit 1; }
  python3 - "$lib" <<'PY'
import csv, glob, sys, collections
f = glob.glob("gpurun_out/r05A_pmc_%s/**/*counter_collection.csv" % sys.argv[1], recursive=True)[0]
rows = list(csv.DictReader(open(f)))
last = sorted(set(r["Dispatch_Id"] for r in rows))[-1]
tot = collections.defaultdict(float)
for r in rows:
    if r["Dispatch_Id"] == last:
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
print("  %s per flush per wave: " % sys.argv[1] + " ".join("%s %.1f" % (k.replace("SQ_", ""), v / 9990 / 8) for k, v in sorted(tot.items())))
PY
done
unset GK_LIB_PATH
for rep in 1 2; do
  for lib in libgkarray_hip.so libgkarray_hip_base.so; do
    GK_LIB_PATH=sketches-py_amd/gkarray_amd/$lib timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 $lib" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
