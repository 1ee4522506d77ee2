# One SQ counter pass over one cfg3 bench step (instruction mix of k_ingest*).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-sq}
D=gpurun_out/$TAG
mkdir -p $D
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY \
  --kernel-include-regex "k_ingest" --output-format csv -d $D -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $D/sq.log 2>&1 || exit $?
python3 - $D <<'PY'
import csv, glob, sys, collections
rows = []
for p in glob.glob(sys.argv[1] + "/*counter_collection.csv"):
    rows += list(csv.DictReader(open(p)))
agg = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
for r in rows:
    agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"]); names[int(r["Dispatch_Id"])] = r["Kernel_Name"][:40]
for d in sorted(agg):
    print(d, names[d], " ".join("%s=%.3g" % (k, v) for k, v in sorted(agg[d].items())))
PY
