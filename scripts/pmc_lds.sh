# LDS / issue counters of k_ingest_small on cfg3 (one --pmc pass each, no tracing)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-lds}
LIB=${2:-libgkarray_hip.so}
export GK_LIB_PATH=$GRAFT_REPO_ROOT/sketches-py_amd/gkarray_amd/$LIB
D=gpurun_out/pmc_$TAG
mkdir -p $D
ARGS="python3 bench.py --steps 1 --warmup 0 --no-cpu"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY \
  --kernel-include-regex "k_ingest" --output-format csv -d $D/p1 -o run -- $ARGS > $D/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES \
  --kernel-include-regex "k_ingest" --output-format csv -d $D/p2 -o run -- $ARGS > $D/p2.log 2>&1 || exit $?
python3 - $D <<'PY'
import csv, collections, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    acc = collections.defaultdict(float); disp = set()
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); disp.add(r["Dispatch_Id"])
    print(f, {k: "%.4g" % (v / len(disp)) for k, v in sorted(acc.items())})
PY
