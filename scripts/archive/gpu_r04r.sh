# Round-4: non-blocking reset (voided deferrals): full suite, cfg3/cfg5
# bench, strong-split proxies, cfg3 kernel trace (the gaps between launches).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
L=sketches-py_amd/gkarray_amd
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; local wl=$2; shift 2
  env "$@" timeout -k 10 200 python bench.py --no-cpu --workload $wl --steps 10 --warmup 3 $BARGS > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-40s %8.3f Gv/s  ms/step %.3f  launch_ms %.3f  frac %.3f' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_full.log 2>&1
rc=$?
log "full -m gpu rc=$rc: $(tail -1 gpurun_out/${TAG}_full.log)"
grep -E "^E  |^FAILED|^ERROR" gpurun_out/${TAG}_full.log | head -20 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -ne 0 ]; then log "abort (rc $rc)"; exit 1; fi
for rep in 1 2; do
  bline cfg3 cfg3 || exit 1
  bline cfg3_r03lib cfg3 GK_LIB_PATH=$L/libgkarray_hip_r03.so || exit 1
done
for S in 500000 250000 125000; do BARGS="--streams $S" bline proxy_S$S cfg3 || exit 1; done
bline cfg2 cfg2 || exit 1
bline cfg5 cfg5 || exit 1
D=gpurun_out/prof_${TAG}_cfg3
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 > $D/bench.log 2>&1
log "cfg3 profile rc=$?"
