# SQ counters of k_ingest_wg alone (tools/wg_alone.py 1: one 10^7-value stream, 9 990 flushes per call),
# one rocprofv3 --pmc pass each, no tracing domains.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r05z}
ARGS="python3 tools/wg_alone.py 1 10000000 2"
i=0
for CNT in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_THREAD_CYCLES_VALU" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_ANY SQ_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_LDS_CMD_FIFO_FULL"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-include-regex "k_ingest_wg" --output-format csv \
    -d gpurun_out/${TAG}_p$i -o run -- $ARGS > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
  echo "pass $i ok"
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float)
for f in sorted(glob.glob("gpurun_out/r05z_p*/**/*counter_collection.csv", recursive=True)):
    rows = list(csv.DictReader(open(f)))
    disp = sorted(set(r["Dispatch_Id"] for r in rows))
    last = disp[-1]  # the last timed call
    for r in rows:
        if r["Dispatch_Id"] == last:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
fl = 9990.0
waves = tot.get("SQ_WAVES", 0)
print("per flush (last call; %d waves in the dispatch incl. the spare workgroups):" % waves)
for k in sorted(tot):
    print("  %-24s %14.0f  per flush %10.1f  per flush per wave(8) %8.1f" % (k, tot[k], tot[k] / fl, tot[k] / fl / 8))
PY
