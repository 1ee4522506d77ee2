# Round-4: the speculative k_stats_long walk -- parity, cfg5 A/B (host walk
# on/off, k_ingest_wg on/off) and a kernel trace with the host walk off.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
bline() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu --workload cfg5 --steps 5 --warmup 2 > gpurun_out/${TAG}_ab.tmp 2>&1 || { log "FAILED: $name"; tail -20 gpurun_out/${TAG}_ab.tmp; return 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_ab.tmp').read().strip().splitlines()[-1]); print('%-36s %7.3f Gv/s  ms/step %.3f  launch_ms %.3f  stats_ms %s' % (sys.argv[1], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline'].get('stats_kernel_ms')))" "$name" | tee -a gpurun_out/${TAG}_ab.txt
}
timeout -k 10 500 python -u -m pytest tests/test_gpu_spec_chain.py tests/test_gpu_hostchains.py tests/test_gpu_configs.py tests/test_gpu_presort.py tests/test_gpu_wg.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
log "tests rc=$rc: $(tail -1 gpurun_out/${TAG}_tests.log)"
grep -E "^E  |^FAILED" gpurun_out/${TAG}_tests.log | head -12 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
for rep in 1 2; do
  bline cfg5_default || exit 1
  bline cfg5_hc0 GK_HOST_CHAINS=0 || exit 1
  bline cfg5_hc0_wg GK_HOST_CHAINS=0 GK_WG=1 || exit 1
done
D=gpurun_out/prof_${TAG}_cfg5
mkdir -p $D
GK_HOST_CHAINS=0 GK_WG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --workload cfg5 --no-cpu --steps 3 --warmup 1 > $D/bench.log 2>&1
log "cfg5 profile rc=$?"
