"""D2H bandwidth on the box: one large pinned copy, and 16 threads copying
2/8/32 MiB chunks on their own streams (host-walked chains' copy pattern)."""
import threading
import time

import torch

N = 1 << 28  # 2 GiB of doubles
x = torch.empty(N, dtype=torch.float64, device="cuda").uniform_()
h = torch.empty(N, dtype=torch.float64, pin_memory=True)
torch.cuda.synchronize()
for rep in range(2):
    t = time.perf_counter()
    h.copy_(x)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
print("one copy: %.1f GB/s" % (N * 8 / dt / 1e9))
for mb in (2, 8, 32):
    for T in (1, 4, 16):
        c = mb << 17
        nchunk = N // c

        def work(tid):
            s = torch.cuda.Stream()
            buf = torch.empty(c, dtype=torch.float64, pin_memory=True)
            with torch.cuda.stream(s):
                for k in range(tid, nchunk, T):
                    buf.copy_(x[k * c:(k + 1) * c], non_blocking=True)
                    s.synchronize()
        t = time.perf_counter()
        th = [threading.Thread(target=work, args=(i,)) for i in range(T)]
        [a.start() for a in th]
        [a.join() for a in th]
        dt = time.perf_counter() - t
        print("chunks %2d MiB x %2d threads: %.1f GB/s" % (mb, T, N * 8 / dt / 1e9), flush=True)
