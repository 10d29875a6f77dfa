"""Decode-side phase times (LFM_DECODE_TIMING) of the bench's config-3 stack.
usage: LFM_DECODE_TIMING=1 python scripts/decode_phases.py"""
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
enc = lfm.Encoder(device=0, num_threads=16)  # owns the .lfm buffer (copy=False)
buf, _ = enc.encode_slab(d, 0, header_version=forced_request(k), nnum=T, copy=False)
buf = bytes(buf)
if os.environ.get("CLOSE_ENC", "0") != "0":  # a reader process has no encoder (bench.py closes it too)
    enc.close()
ref = d.cpu().numpy().view(np.uint16)
for it in range(3):
    img = None  # free the previous result first (its unmap is not the decode's)
    t0 = time.perf_counter()
    img = lfm.decode(buf)
    ms = (time.perf_counter() - t0) * 1e3
    print("decode %d: %.1f ms, exact %s, payload %.1f MB" % (it, ms, bool((img.reshape(ref.shape) == ref).all()),
                                                          len(buf) / 1e6), flush=True)
