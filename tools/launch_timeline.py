"""Where a k_ingest_small launch spends its wall time (timeline build only).

Run on a GPU box after
    make -C sketches-py_amd/csrc variant VNAME=tl VFLAGS=-DGK_TIMELINE
as  python3 tools/launch_timeline.py [S[:L[:XOFF_GB]] ...]   (cfg3 batches of S streams of L values,
    default 1000, optionally placed XOFF_GB GiB into a larger device buffer)
Loads libgkarray_hip_tl.so (GK_LIB_PATH), runs warm-up steps (reset + fused
ingest + quantiles), then one recorded step, and prints from the
s_memrealtime stamps (100 MHz, chip-wide) of every wave (start, stats role
done, end) and every stream (start, end): the waves' start spread, the
stats role, the stream completion rate over the launch, per-stream wave time
by phase, the tail after the last stream was handed out, and the shader clock
(s_memtime over s_memrealtime) over each wave's life.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "sketches-py_amd", "gkarray_amd", "libgkarray_hip_tl.so")
os.environ.setdefault("GK_LIB_PATH", LIB)
sys.path.insert(0, os.path.join(ROOT, "sketches-py_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

MAXW, MAXS = 16384, 1 << 20


def pct(a, qs=(0, 1, 10, 50, 90, 99, 100)):
    return " ".join("p%d=%.1f" % (q, np.percentile(a, q)) for q in qs)


def wg_clock(arg, lib, dev):
    """k_ingest_wg's workgroups: wall time, flushes, us per flush and shader
    clock per workgroup.  "wg:cfg5": the bench's cfg5 batch (everything
    beside the workgroups); "wg:S": S lognormal streams of 10^7 values alone."""
    from bench import make_zipf_input
    from gkarray_amd import StreamSet
    what = arg.split(":")[1] if ":" in arg else "cfg5"
    if what == "cfg5":
        x, offs = make_zipf_input(100_000, 5, dev)
    else:
        S, L = int(what), 10_000_000
        g = torch.Generator(device=dev).manual_seed(5)
        x = torch.exp(torch.randn(S * L, device=dev, dtype=torch.float64, generator=g))
        offs = torch.arange(S + 1, device=dev, dtype=torch.int64) * L
    ss = StreamSet(offs.numel() - 1, 0.001, device=dev)
    for _ in range(int(os.environ.get("TL_WARM", "4"))):
        ss.reset()
        ss.ingest(x, offs, quantiles=[0.5, 0.9, 0.99])
    torch.cuda.synchronize()
    wg = np.zeros(5 * 64, dtype=np.uint64)
    assert lib.gk_tl_wg_read(wg.ctypes.data_as(ctypes.c_void_p)) == 0
    w = wg.reshape(-1, 5).astype(np.int64)
    w = w[(w[:, 0] > 0) & (w[:, 4] > 0)]
    dur = (w[:, 2] - w[:, 0]) / 100.0
    clk = (w[:, 3] - w[:, 1]) / np.maximum(w[:, 2] - w[:, 0], 1) * 100.0
    fl = w[:, 4]
    print("%s (%s warm-up steps): %d workgroups with flushes" % (arg, os.environ.get("TL_WARM", "4"), len(w)))
    order = np.argsort(-fl)
    cl = np.zeros(2, dtype=np.uint64)
    assert lib.gk_tl_call_read(cl.ctypes.data_as(ctypes.c_void_p)) == 0
    t0 = int(cl[0])  # the call's first kernel (k_lengths)
    st_us, en_us = (w[:, 0] - t0) / 100.0, (w[:, 2] - t0) / 100.0
    print("  the call: k_lengths start -> k_query_list (the join) %.0f us; first workgroup start %.0f us"
          % ((int(cl[1]) - t0) / 100.0, st_us.min()))
    print("  flushes   start us   end us   wall us   us/flush   clock MHz   (the 12 longest chains; times from the call's first kernel)")
    for i in order[:12]:
        print("  %7d %9.0f %8.0f %9.0f %10.3f %11.0f" % (fl[i], st_us[i], en_us[i], dur[i], dur[i] / fl[i], clk[i]))
    print("  workgroup start us:", pct(st_us))
    print("  workgroup end us:  ", pct(en_us))
    print("  clock MHz over all workgroups:", pct(clk))
    del ss, x, offs
    torch.cuda.empty_cache()


def main():
    from bench import make_input
    from gkarray_amd import StreamSet
    dev = torch.device("cuda", 0)
    lib = ctypes.CDLL(os.environ["GK_LIB_PATH"])
    for arg in sys.argv[1:] or ["125000", "1000000"]:
        if arg.startswith("wg"):
            wg_clock(arg, lib, dev)
            continue
        f = arg.split(":")
        S, L = int(f[0]), int(f[1]) if len(f) > 1 else 1000
        x, offs = make_input(S, L, 3, dev, "pareto")
        if len(f) > 2:  # the same values at another address: XOFF_GB GiB into a bigger buffer
            off = int(float(f[2]) * (1 << 30)) // 8
            big = torch.empty(off + x.numel(), dtype=x.dtype, device=dev)
            big[off:] = x
            x = big[off:]
        ss = StreamSet(S, 0.01, device=dev)
        for _ in range(int(os.environ.get("TL_WARM", "4"))):  # warm-up steps before the recorded one
            ss.reset()
            ss.ingest(x, offs, quantiles=[0.5, 0.9, 0.99])
        torch.cuda.synchronize()
        wave = np.zeros(5 * MAXW, dtype=np.uint64)
        sb = np.zeros(MAXS, dtype=np.uint64)
        se = np.zeros(MAXS, dtype=np.uint64)
        assert lib.gk_tl_read(wave.ctypes.data_as(ctypes.c_void_p), sb.ctypes.data_as(ctypes.c_void_p),
                              se.ctypes.data_as(ctypes.c_void_p)) == 0
        w = wave.reshape(-1, 5).astype(np.int64)
        w = w[w[:, 0] > 0]
        sbeg = sb[:S].astype(np.int64)
        send = se[:S].astype(np.int64)
        ok = (sbeg > 0) & (send > 0)
        t0 = w[:, 0].min()
        us = lambda a: (a - t0) / 100.0  # 100 MHz ticks -> us
        ws, wr, we = us(w[:, 0]), us(w[:, 1]), us(w[:, 2])
        b, e = us(sbeg[ok]), us(send[ok])
        T = we.max()
        print("%s (%s warm-up steps): %d waves, %d streams stamped; launch (first wave start -> last wave end) %.1f us"
              % (arg, os.environ.get("TL_WARM", "4"), len(w), ok.sum(), T))
        print("  wave start        ", pct(ws))
        bidx = np.nonzero(wave.reshape(-1, 5)[:, 0] > 0)[0]
        late = ws > 100.0
        if late.any():
            print("  late waves (start > 100 us): %d, blockIdx %s, their stats-role end %s, end %s"
                  % (late.sum(), pct(bidx[late]), pct(wr[late]), pct(we[late])))
        # the shader clock over each wave's life: s_memtime ticks / s_memrealtime ticks x 100 MHz
        clk = (w[:, 4] - w[:, 3]) / np.maximum(w[:, 2] - w[:, 0], 1) * 100.0
        print("  shader clock MHz  ", pct(clk))
        stat = wr - ws > 1.0
        if stat.any():
            print("  stats role end     (%d waves) %s" % (stat.sum(), pct(wr[stat])))
        print("  wave end          ", pct(we))
        print("  stream start      ", pct(b))
        print("  stream end        ", pct(e))
        last_start = b.max()
        print("  last stream start %.1f us; after it: %.1f us to the last wave end (%.1f%% of the launch)" %
              (last_start, T - last_start, 100.0 * (T - last_start) / T))
        # completion rate over the launch in 20 bins; per-stream wave time by bin (by start)
        nb = 20
        edges = np.linspace(0, T, nb + 1)
        cnt, _ = np.histogram(e, edges)
        dur = e - b
        idx = np.clip(np.digitize(b, edges) - 1, 0, nb - 1)
        print("  bin(us)   streams done   rate(/us)   median stream time (us, by start)")
        for i in range(nb):
            d = dur[idx == i]
            print("  %6.0f-%6.0f %8d %10.1f %10.1f" % (edges[i], edges[i + 1], cnt[i], cnt[i] / (edges[i + 1] - edges[i]),
                                                        np.median(d) if len(d) else float("nan")))
        del ss, x, offs
        big = None
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
