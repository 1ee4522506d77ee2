"""Where k_ingest_small spends its time, by section (profiling build only).

Run on a GPU box after `make -C sketches-py_amd/csrc prof`:
    python3 tools/prof_sections.py [--workload cfg3|cfg2] [--streams S]
Loads libgkarray_hip_prof.so (GK_LIB_PATH), runs one bench step (reset +
fused ingest+quantiles) untimed, then one profiled step, and prints the
s_memtime cycles accumulated per section over all waves (lane 0 marks, so the
numbers are per-wave latencies summed; the shares are what matters).
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "sketches-py_amd", "gkarray_amd", "libgkarray_hip_prof.so")
os.environ.setdefault("GK_LIB_PATH", LIB)
sys.path.insert(0, os.path.join(ROOT, "sketches-py_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

SECTIONS = ["stream setup (header, table load)", "gap search", "counts (zero, atomics, max gap)",
            "entries + carry + scan", "keeps + per-gap info", "rank loop + emit", "bitonic sort + emit",
            "pad + end of flush", "between flushes (T, next flush setup)", "leftover, quantiles, write-back",
            "next flush's values (prefetch wait)", "between flushes, a wave's first stream"]

SECTIONS_WG = ["stream setup + loop top", "batch load + next-batch prefetch", "gap search + counts",
               "carry walk", "scan + per-gap bases + keeps", "member stores (unsorted)",
               "rank + place + pad", "end of flush", "-", "write-back", "crowded-gap sort", "-"]

SECTIONS_BIG = ["stream setup (header, table load)", "gap search", "counts (zero, atomics, max gap)",
                "carry walk (rounds)", "sums + scan + keeps", "rank loop + emit", "bitonic sort + emit",
                "pad + end of flush", "between flushes", "leftover, quantiles, write-back", "-", "-"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cfg3", choices=["cfg3", "cfg2", "long", "wg", "cfg5"])
    ap.add_argument("--streams", type=int, default=0)
    ap.add_argument("--per-wave", action="store_true",
                    help="wg: per-wave work / barrier-wait split of every stretch of the flush (GK_WMARK)")
    a = ap.parse_args()
    from bench import make_input, make_zipf_input
    from gkarray_amd import StreamSet
    S, L, dist_name = {"cfg3": (1_000_000, 1000, "pareto"), "cfg2": (100_000, 10_000, "lognormal"),
                       "long": (64, 1_000_000, "lognormal"), "wg": (64, 1_000_000, "lognormal"),
                       "cfg5": (100_000, 0, "zipf")}[a.workload]
    S = a.streams or S
    dev = torch.device("cuda", 0)
    if a.workload == "cfg5":  # the bench's cfg5 batch: every k_ingest_wg stream beside everything else
        x, offs = make_zipf_input(S, 5, dev)
    else:
        x, offs = make_input(S, L, 3, dev, dist_name)
    # "long": eps=0.001 streams of 1M values in the 2048 class (k_ingest<2048>,
    # sections of flush_wave: SECTIONS_BIG)
    # "wg": the same streams through k_ingest_wg (GK_WG=1; GK_WG_PRESORT from
    # the environment), sections of flush_wg: SECTIONS_WG
    eps = 0.001 if a.workload in ("long", "wg", "cfg5") else 0.01
    global SECTIONS
    if a.workload == "long":
        SECTIONS = SECTIONS_BIG
    if a.workload in ("wg", "cfg5"):
        os.environ["GK_WG"] = "1"
        SECTIONS = SECTIONS_WG
    ss = StreamSet(S, eps, device=dev)
    lib = ctypes.CDLL(os.environ["GK_LIB_PATH"])
    acc = (ctypes.c_ulonglong * 12)()
    for it in range(2):
        ss.reset()
        torch.cuda.synchronize()
        assert lib.gk_prof_reset() == 0
        ss.ingest(x, offs, quantiles=[0.5, 0.9, 0.99])
        torch.cuda.synchronize()
    assert lib.gk_prof_read(acc) == 0
    if a.per_wave:
        W, N = 8, 16
        wacc = (ctypes.c_ulonglong * (W * N))()
        assert lib.gk_wprof_read(wacc) == 0
        names = ["between flushes (loads)", "setup (zero, g/d loads)", "gap search", "count atomics",
                 "count barrier", "carry walk", "carry barrier", "carry DPP rounds x1000", "scan barrier",
                 "totals + placement", "placement barrier", "values + pad", "end barrier",
                 "loop top up to the batch copy (incl. its wait)"]
        flushes = S * (L // 1001)
        if a.workload == "cfg5":  # the workgroup streams: >= 256 flushes, the 64 longest (GK_WG_MAX)
            lens = sorted(((offs[1:] - offs[:-1]).cpu().tolist()), reverse=True)
            wl = [n for n in lens if n // 1001 >= 256][:64]
            flushes = sum(n // 1001 for n in wl)
        print("per-wave stretches, cycles per flush (%d flushes): wave0 / min / max over the 8 waves" % flushes)
        for i, nm in enumerate(names):
            v = [wacc[w * N + i] / flushes for w in range(W)]
            print("  %2d %-28s %8.0f %8.0f %8.0f" % (i, nm, v[0], min(v), max(v)))
        print("  total per flush (wave 0, cycles): %.0f" % (sum(wacc[i] for i in range(N) if i != 7) / flushes))
    tot = sum(acc)
    print("workload %s: %d streams x %d values, total %.3e cycles (sum over waves)" % (a.workload, S, L, tot))
    for i, name in enumerate(SECTIONS):
        if acc[i]:
            print("  %2d %-36s %6.1f%%  %.3e" % (i, name, 100.0 * acc[i] / tot, acc[i]))


if __name__ == "__main__":
    main()
