# Round-4: new defaults (k_ingest_wg on, presorted; host chains off):
# the full GPU suite, cfg5 A/B of the wg rank unroll / presort, cfg3 bench,
# kernel-trace profiles of cfg3 and cfg5.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
L=sketches-py_amd/gkarray_amd
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; local wl=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu --workload $wl --steps 5 --warmup 2 > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-40s %7.3f Gv/s  ms/step %.3f  launch_ms %.3f  stats_ms %s' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline'].get('stats_kernel_ms')))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_full.log 2>&1
rc=$?
log "full -m gpu rc=$rc: $(tail -1 gpurun_out/${TAG}_full.log)"
grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_full.log | head -20 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
GK_WG_PRESORT=0 timeout -k 10 200 python tools/prof_sections.py --workload wg > gpurun_out/${TAG}_sections_ps0.txt 2>&1 || { log "prof failed"; exit 1; }
log "== wg sections, GK_WG_PRESORT=0"; grep -v amdgpu.ids gpurun_out/${TAG}_sections_ps0.txt | tee -a gpurun_out/${TAG}_ab.txt
for rep in 1 2; do
  bline cfg5_default cfg5 || exit 1
  bline cfg5_nopresort cfg5 GK_WG_PRESORT=0 || exit 1
  bline cfg5_nopresort_rk8 cfg5 GK_WG_PRESORT=0 GK_LIB_PATH=$L/libgkarray_hip_rk8.so || exit 1
  bline cfg5_hc1 cfg5 GK_HOST_CHAINS=1 || exit 1
done
bline cfg3 cfg3 || exit 1
bline cfg2 cfg2 || exit 1
D=gpurun_out/prof_${TAG}_cfg5
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > $D/bench.log 2>&1
log "cfg5 profile rc=$?"
D=gpurun_out/prof_${TAG}_cfg3
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 > $D/bench.log 2>&1
log "cfg3 profile rc=$?"
