"""Device allocations per bench step, from a rocprofv3 run with
--memory-allocation-trace --kernel-trace (scripts/gpu_round.sh): the steps are
delimited by the bench's k_reset launches (every step starts with reset();
`resets` per step).  Prints one line per step: allocation calls and bytes.

Usage: alloc_steps.py DIR RESETS_PER_STEP [TIMED_STEPS]"""
import csv
import glob
import sys


def rows(d, name):
    out = []
    for p in glob.glob("%s/**/*%s*.csv" % (d, name), recursive=True):
        out.extend(csv.DictReader(open(p)))
    return out


def main(d, per, timed=None):
    k = sorted(int(r["Start_Timestamp"]) for r in rows(d, "kernel_trace") if r["Kernel_Name"].startswith("k_reset"))
    starts = k[::per]
    allocs = [r for r in rows(d, "memory_allocation_trace")
              if "FREE" not in r.get("Operation", "").upper()]
    print("%d steps (%d k_reset launches), %d allocation records" % (len(starts), len(k), len(allocs)))
    bounds = starts + [float("inf")]
    lines = []
    for i in range(len(starts)):
        a, b = bounds[i], bounds[i + 1]
        sel = [r for r in allocs if a <= int(r["Start_Timestamp"]) < b]
        nbytes = sum(int(r.get("Allocation_Size", 0) or 0) for r in sel)
        tag = ""
        if timed is not None and i >= len(starts) - timed:
            tag = "  (timed)"
        lines.append("step %d: %d allocations, %d bytes%s" % (i, len(sel), nbytes, tag))
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else None)
