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


def main():
    from bench import make_input
    from gkarray_amd import StreamSet
    dev = torch.device("cuda", 0)
    lib = ctypes.CDLL(os.environ["GK_LIB_PATH"])
    for arg in sys.argv[1:] or ["125000", "1000000"]:
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
