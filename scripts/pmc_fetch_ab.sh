# FETCH_SIZE of k_ingest_small (the bench's dominant kernel) per env config:
# one PMC pass each (no tracing domain), 1 bench step.
# Usage: pmc_fetch_ab.sh TAG "ENV1=.. ENV2=.." ...   -> gpurun_out/TAG_fetch.txt
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1; shift
i=0
for cfg in "$@"; do
  i=$((i+1))
  D=gpurun_out/${TAG}_f$i
  env $cfg timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_ingest_small" --output-format csv \
    -d $D -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $D.log 2>&1 || { echo "FAILED: $cfg"; tail -5 $D.log; exit 1; }
  python3 - "$cfg" "$D" <<'PY' | tee -a gpurun_out/${TAG}_fetch.txt
import csv, glob, sys
from collections import defaultdict
agg = defaultdict(float)
for p in glob.glob(sys.argv[2] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if r["Counter_Name"] == "FETCH_SIZE" and "k_ingest_small" in r["Kernel_Name"]:
            agg[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
v = max(agg.values()) if agg else float("nan")
print("%-60s FETCH_SIZE %.3f GB (x2 corrected %.3f GB) over %d dispatch(es)" % (sys.argv[1], v * 1024 / 1e9, 2 * v * 1024 / 1e9, len(agg)))
PY
done
