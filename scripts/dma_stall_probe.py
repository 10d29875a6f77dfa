"""Is the slow first host->device copy of a decode a platform effect?  Times a
32 MiB pinned host->device copy (torch, no lfm code) after host-side events:
nothing, freeing a touched 537 MB array (munmap), allocating and touching one,
a 0.35 s sleep, and a 64 KiB copy ahead of the big one.
usage: python scripts/dma_stall_probe.py"""
import time

import numpy as np
import torch

torch.cuda.set_device(0)
N = 32 << 20
pinned = torch.empty(N, dtype=torch.uint8).pin_memory()
small = torch.empty(64 << 10, dtype=torch.uint8).pin_memory()
dev = torch.empty(N, dtype=torch.uint8, device="cuda")
dsmall = torch.empty(64 << 10, dtype=torch.uint8, device="cuda")
IMG = 2048 * 2048 * 64


def copy(src, dst):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3


def report(tag, xs):
    print("%-34s %s" % (tag, " ".join("%.2f" % x for x in xs)), flush=True)


report("back to back", [copy(pinned, dev) for _ in range(6)])
r = []
for _ in range(5):
    a = np.ones(IMG, np.uint16)
    del a
    r.append(copy(pinned, dev))
report("after alloc+touch+free", r)
r = []
keep = None
for _ in range(5):
    a = np.ones(IMG, np.uint16)
    r.append(copy(pinned, dev))
    keep = a
report("after alloc+touch (kept)", r)
del keep
r = []
for _ in range(5):
    time.sleep(0.35)
    r.append(copy(pinned, dev))
report("after 0.35 s sleep", r)
r, s = [], []
for _ in range(5):
    a = np.ones(IMG, np.uint16)
    del a
    s.append(copy(small, dsmall))
    r.append(copy(pinned, dev))
report("after free: 64 KiB copy", s)
report("after free: then 32 MiB", r)
r = []
for _ in range(5):
    a = np.ones(IMG, np.uint16)
    del a
    time.sleep(0.05)
    r.append(copy(pinned, dev))
report("after free + 50 ms", r)
r = []
for _ in range(5):
    a = np.ones(IMG, np.uint16)
    del a
    time.sleep(0.2)
    r.append(copy(pinned, dev))
report("after free + 200 ms", r)
