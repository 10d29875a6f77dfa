"""Does the first upload of a decode stall after the GPU sat idle?  Decodes the
bench's config-3 .lfm back to back, then with pauses (sleep / a CPU compare)
between the calls; LFM_DECODE_TIMING=1 prints each decode's timeline.
usage: LFM_DECODE_TIMING=1 python scripts/decode_idle_probe.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lightfieldmicroscopy_pc-bzip2_amd"))
import lfm  # noqa: E402
from lfm.shard import forced_request  # noqa: E402

X, Y, Z, T = 2048, 2048, 64, 15
torch.cuda.set_device(0)
lfm.require_gpu()
lfm.set_family("angle")
d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
lfm.synth_device(d, X, Y, Z, T, t_index=0, idx0=0, seed=0x4C464D03)
torch.cuda.synchronize()
k, _ = lfm.select_device(d[0], X, Y, T, "angle")
enc = lfm.Encoder(device=0, num_threads=16)
buf, _ = enc.encode_slab(d, 0, header_version=forced_request(k), nnum=T, copy=False)
buf = bytes(buf)
enc.close()
out = np.empty(X * Y * Z, np.uint16)  # one destination, already faulted in after the first call


def one(tag):
    t0 = time.perf_counter()
    img = lfm.decode(buf)
    print("%s: %.1f ms" % (tag, (time.perf_counter() - t0) * 1e3), flush=True)
    return img


ref = d.cpu().numpy().view(np.uint16).reshape(-1)
img = one("warm")
for i in range(2):  # the bench's pattern: compare, free, decode into a fresh array
    ok = bool(np.array_equal(img.reshape(-1), ref))
    del img
    img = one("after compare + free %d (exact %s)" % (i, ok))
for i in range(2):  # free only
    del img
    img = one("after free %d" % i)
for i in range(2):  # compare only (the old array is freed after the decode)
    ok = bool(np.array_equal(img.reshape(-1), ref))
    img = one("after compare %d" % i)
for i in range(2):  # sleep as long as a compare takes
    time.sleep(0.35)
    img = one("after 0.35 s sleep %d" % i)
