"""Device -> host rates behind the decode's download: torch (hipMemcpyAsync)
device -> pinned, pinned -> pageable host memcpy (numpy, one thread), for a
268 MB piece (one decode chunk of config 3).
usage: python scripts/d2h_rate_probe.py"""
import time

import numpy as np
import torch

torch.cuda.set_device(0)
N = 268 << 20
dev = torch.empty(N, dtype=torch.uint8, device="cuda")
dev.fill_(7)
pin = torch.empty(N, dtype=torch.uint8).pin_memory()
pin32 = torch.empty(32 << 20, dtype=torch.uint8).pin_memory()


def t(f, reps=5):
    xs = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f()
        torch.cuda.synchronize()
        xs.append((time.perf_counter() - t0) * 1e3)
    return min(xs), float(np.median(xs))


def gbs(ms, n=N):
    return n / ms / 1e6


mn, md = t(lambda: pin.copy_(dev, non_blocking=True))
print("D2H pinned 268 MB (hipMemcpyAsync): min %.2f ms (%.1f GB/s), median %.2f" % (mn, gbs(mn), md), flush=True)
mn, md = t(lambda: pin32.copy_(dev[:32 << 20], non_blocking=True))
print("D2H pinned 32 MB: min %.3f ms (%.1f GB/s)" % (mn, gbs(mn, 32 << 20)), flush=True)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
h = N // 2


def two():
    with torch.cuda.stream(s1):
        pin[:h].copy_(dev[:h], non_blocking=True)
    with torch.cuda.stream(s2):
        pin[h:].copy_(dev[h:], non_blocking=True)


mn, md = t(two)
print("D2H pinned 268 MB as two streams: min %.2f ms (%.1f GB/s)" % (mn, gbs(mn)), flush=True)
dst = np.empty(N, np.uint8)
dst[:] = 1
src = pin.numpy()
mn, md = t(lambda: np.copyto(dst, src))
print("host memcpy pinned -> touched pageable (1 thread): min %.2f ms (%.1f GB/s)" % (mn, gbs(mn)), flush=True)
