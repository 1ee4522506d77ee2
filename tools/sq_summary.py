"""Per-launch SQ counters of k_ingest_small from scripts/pmc_sq.sh output dirs,
per flush (1e7 flushes per cfg3 launch) and LDS share.  Usage: sq_summary.py TAG [TAG2 ...]
(KRX in the environment: another kernel name, e.g. k_ingest_wg)"""
import csv
import glob
import os
import sys

FLUSHES = 1e7


def load(tag):
    agg = {}
    for f in glob.glob("gpurun_out/%s_p*/**/*counter_collection.csv" % tag, recursive=True):
        for r in csv.DictReader(open(f)):
            if os.environ.get("KRX", "k_ingest_small") in r["Kernel_Name"]:
                agg.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: v[-1] for k, v in agg.items()}


tags = sys.argv[1:]
data = [load(t) for t in tags]
keys = sorted(set().union(*[d.keys() for d in data]))
print("%-26s" % "counter" + "".join("%16s" % t for t in tags))
for k in keys:
    print("%-26s" % k + "".join("%16.4g" % d.get(k, float("nan")) for d in data))
print("%-26s" % "VALU/flush" + "".join("%16.1f" % (d.get("SQ_INSTS_VALU", 0) / FLUSHES) for d in data))
print("%-26s" % "SALU/flush" + "".join("%16.1f" % (d.get("SQ_INSTS_SALU", 0) / FLUSHES) for d in data))
print("%-26s" % "LDS/flush" + "".join("%16.1f" % (d.get("SQ_INSTS_LDS", 0) / FLUSHES) for d in data))
print("%-26s" % "LDS busy / SQ cycles" + "".join(
    "%16.3f" % (d.get("SQ_LDS_IDX_ACTIVE", 0) / 256 / max(d.get("SQ_CYCLES", 1) / 32, 1)) for d in data))
print("%-26s" % "bank conflict share" + "".join(
    "%16.3f" % (d.get("SQ_LDS_BANK_CONFLICT", 0) / max(d.get("SQ_LDS_IDX_ACTIVE", 1), 1)) for d in data))
