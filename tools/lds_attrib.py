"""LDS cost attribution table from scripts/lds_attrib.sh's PMC passes.

Each attribution build (-DGK_DUP=1<<g) issues one access group of the
small-class flush twice; its counter deltas against the product build are
that group's LDS instructions, LDS-array cycles and bank-conflict cycles
(per flush: the launch's counts / flushes).  Usage:
    python3 tools/lds_attrib.py gpurun_out TAG base.so dupN.so ...
"""
import csv
import glob
import sys
from collections import defaultdict

GROUPS = {
    1: "search levels S=64..8 (4 x 2 ds_read_b64)",
    2: "search levels S=4..1 (3 x 2 ds_read_b64)",
    3: "count atomics' addresses (as ds_read_b32)",
    4: "entry reads (tgd b128+b64, tv 2xb64, counts 2xb32)",
    5: "kept-entry stores (tv + tgd b64, 2 entries)",
    6: "member stores (mv b64 + inf pad)",
    7: "per-gap record reads (int2, 2 values)",
    8: "emit stores (tv + tgd b64, 2 values)",
    9: "in-gap rank loop reads (mv b64)",
    10: "first-flush stores (tv + tgd b64)",
    11: "per-gap record stores (int2 x 2)",
    12: "pad + count zeroing stores",
}
FLUSHES = 1.0e7  # cfg3: 10^6 streams x ~10 flushes per launch


def load(root, tag, lib):
    agg = defaultdict(lambda: defaultdict(float))
    for p in glob.glob(f"{root}/{tag}_{lib[:-3]}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if "k_ingest_small" in r["Kernel_Name"]:
                agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    if not agg:
        return None
    return agg[max(agg)]  # the last launch (warm)


def main():
    root, tag, base, *libs = sys.argv[1:]
    b = load(root, tag, base)
    cols = ["SQ_INSTS_LDS", "SQ_LDS_IDX_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_ADDR_CONFLICT", "SQ_INSTS_VALU"]
    print("per flush (%.0e flushes per launch)" % FLUSHES)
    print("%-58s" % "build" + "".join("%14s" % c.replace("SQ_", "") for c in cols))
    print("%-58s" % base + "".join("%14.1f" % (b[c] / FLUSHES) for c in cols))
    for lib in libs:
        d = load(root, tag, lib)
        if d is None:
            print(lib, "missing")
            continue
        g = int(lib.split("dup")[1].split(".")[0]) if "dup" in lib else 0
        name = GROUPS.get(g, lib)
        print("%-58s" % ("+%d %s" % (g, name))[:58] + "".join("%14.1f" % ((d[c] - b[c]) / FLUSHES) for c in cols))


if __name__ == "__main__":
    main()
