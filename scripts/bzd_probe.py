"""Kernel-time probe of the GPU bzip2 decode on the bench's config-3 stack:
encode once, decode `reps` times (errors tolerated: the LFM_BZD_PROBE
libraries under exp/ skip decode work on purpose and fail the CRC).  Run
under rocprofv3 --kernel-trace --stats for the per-kernel times.
usage: [LFM_LIB=...] python scripts/bzd_probe.py [reps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lightfieldmicroscopy_pc-bzip2_amd"))
import lfm  # noqa: E402
from lfm.shard import forced_request  # noqa: E402

X, Y, Z, T = 2048, 2048, 64, 15
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
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
for it in range(reps):
    t0 = time.perf_counter()
    try:
        lfm.decode(buf)
        ok = True
    except Exception as e:  # noqa: BLE001
        ok = "error: %s" % str(e)[:60]
    print("decode %d: %.1f ms, %s" % (it, (time.perf_counter() - t0) * 1e3, ok), flush=True)
