# spec-chain fix (failed superstep walked alone, then resume): spec/wg tests, wg_alone S=23,
# cfg5 A/B over the wave priorities of k_stats_long (GK_SL_PRIO) and k_ingest_wg (GK_WG_PRIO).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05w}
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('%-34s %8.2f Gv/s ms/step %.4f launch %.4f frac %.4f' % (sys.argv[2], d['value']/1e9, d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac']))" "$@"; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_spec_chain.py tests/test_gpu_wg.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/${TAG}_pytest.log | head -20; exit 1; fi
for S in 23; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_S$S -o run -- \
    python3 tools/wg_alone.py $S > gpurun_out/${TAG}_S$S.log 2>&1 || { tail -5 gpurun_out/${TAG}_S$S.log; exit 1; }
  grep "per flush" gpurun_out/${TAG}_S$S.log
  f=$(find gpurun_out/${TAG}_S$S -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'wg' in r['Name'] or 'stats_long' in r['Name']:
        print('   %-40s calls %s avg %.2f ms max %.2f ms' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e6, float(r['MaxNs'])/1e6))
"
done
for rep in 1 2; do
  for pr in "1 0" "0 0" "1 1" "0 1"; do
    set -- $pr
    GK_SL_PRIO=$1 GK_WG_PRIO=$2 timeout -k 10 300 python bench.py --workload cfg5 --no-cpu --steps 10 --warmup 2 > gpurun_out/${TAG}.tmp 2>&1 || { tail -5 gpurun_out/${TAG}.tmp; exit 1; }
    line gpurun_out/${TAG}.tmp "cfg5 SL_PRIO=$1 WG_PRIO=$2" | tee -a gpurun_out/${TAG}_ab.txt
  done
done
