# k_ingest_wg alone: S long streams (10^7 values) and nothing else; kernel trace per S.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05u}
for S in 1 8 23 64; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_S$S -o run -- \
    python3 tools/wg_alone.py $S > gpurun_out/${TAG}_S$S.log 2>&1 || { tail -5 gpurun_out/${TAG}_S$S.log; exit 1; }
  grep "per flush" gpurun_out/${TAG}_S$S.log
  f=$(find gpurun_out/${TAG}_S$S -name '*kernel_stats.csv' | head -1)
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    if 'wg' in r['Name'] or 'stats_long' in r['Name'] or 'presort' in r['Name']:
        print('   %-40s calls %s avg %.2f ms max %.2f ms' % (r['Name'][:40], r['Calls'], float(r['AverageNs'])/1e6, float(r['MaxNs'])/1e6))
"
done
