# Per-kernel totals (rocprofv3 --stats) of one bench configuration over the listed builds.
# Usage: gpu_r6_kstats.sh TAG "bench args" lib1 [lib2 ...]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
L=sketches-py_amd/gkarray_amd
for lib in "$@"; do
  n=${lib%.so}; n=${n#libgkarray_hip}; n=${n#_}; [ -z "$n" ] && n=prod
  GK_LIB_PATH=$L/$lib timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_${n}_ks -o run -- \
    python3 bench.py --no-cpu $ARGS > gpurun_out/${TAG}_${n}_ks.log 2>&1 || { echo "failed $lib"; tail -5 gpurun_out/${TAG}_${n}_ks.log; exit 1; }
  f=$(find gpurun_out/${TAG}_${n}_ks -name "*kernel_stats.csv" | head -1)
  echo "== $lib: $(tail -1 gpurun_out/${TAG}_${n}_ks.log | cut -c1-100)"
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
rows.sort(key=lambda r:-float(r['TotalDurationNs']))
for r in rows[:14]: print('%-60s %6s calls %10.3f ms total %9.1f us avg' % (r['Name'][:60], r['Calls'], float(r['TotalDurationNs'])/1e6, float(r['AverageNs'])/1e3))
"
done
