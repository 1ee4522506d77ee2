# Round-4 evidence run on the current library: GPU suite, smoke, the stamped
# PMC traffic profile of cfg3 (scripts/profile_cfg3.sh), the default bench
# line (with the CPU baseline), the other workloads' lines, SQ counters.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
log() { echo "$@" | tee -a gpurun_out/${TAG}_ab.txt; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?
log "full -m gpu rc=$rc: $(tail -1 gpurun_out/${TAG}_pytest_gpu.log)"
grep -E "^FAILED|^ERROR" gpurun_out/${TAG}_pytest_gpu.log | head -20 | tee -a gpurun_out/${TAG}_ab.txt
if [ $rc -gt 1 ]; then log "abort (rc $rc)"; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
log "smoke rc=$?: $(tail -1 gpurun_out/${TAG}_smoke.log)"
timeout -k 10 900 bash scripts/profile_cfg3.sh $TAG > gpurun_out/${TAG}_profile.log 2>&1
log "profile_cfg3 rc=$?: $(tail -1 gpurun_out/${TAG}_profile.log | cut -c1-200)"
cp gpurun_out/prof_$TAG/pmc_traffic.json profiles/pmc_traffic.json 2>/dev/null && log "stamped pmc_traffic.json"
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench_cfg3.json 2> gpurun_out/${TAG}_bench_cfg3.err
log "bench default rc=$?: $(tail -1 gpurun_out/${TAG}_bench_cfg3.json | cut -c1-400)"
for wl in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu > gpurun_out/${TAG}_bench_$wl.json 2> gpurun_out/${TAG}_bench_$wl.err
  log "bench $wl rc=$?: $(tail -1 gpurun_out/${TAG}_bench_$wl.json | cut -c1-200)"
done
timeout -k 10 300 python bench.py --workload cfg4 --virtual-shards 8 --no-cpu > gpurun_out/${TAG}_bench_cfg4_k8.json 2> gpurun_out/${TAG}_bench_cfg4_k8.err
log "bench cfg4 x8 rc=$?: $(tail -1 gpurun_out/${TAG}_bench_cfg4_k8.json | cut -c1-200)"
bash scripts/pmc_sq.sh ${TAG}_sq > gpurun_out/${TAG}_sq.log 2>&1 && python3 tools/sq_summary.py ${TAG}_sq > gpurun_out/${TAG}_sq_summary.txt 2>&1
log "sq rc=$?"
