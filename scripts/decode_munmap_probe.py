"""Which host event before a decode stalls its first DMA?  With
LFM_DECODE_DMA_PROBE=1 each decode prints the time of a 64 KiB staged SDMA
upload at its entry.  Cases: decode right after a decode; after freeing an
unrelated 537 MB array; after freeing the previous decode's output.
usage: LFM_DECODE_DMA_PROBE=1 python scripts/decode_munmap_probe.py"""
import os
import sys

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


def tag(s):
    print("-- " + s, file=sys.stderr, flush=True)


keep = [lfm.decode(buf)]
for i in range(2):
    tag("decode right after a decode (outputs kept)")
    keep.append(lfm.decode(buf))
mode = os.environ.get("REF", "cpu")
tag("reference copy: " + mode)
if mode == "cpu":
    ref = d.cpu().numpy().view(np.uint16).reshape(-1)  # (torch: device -> pageable host)
elif mode == "host":
    ref = np.empty(X * Y * Z, np.uint16)  # (no device copy: the decode's own output as the reference)
    ref[:] = keep[0].reshape(-1)
elif mode == "pinned":
    ref = torch.empty(d.shape, dtype=d.dtype).pin_memory()
    ref.copy_(d)
    ref = ref.numpy().view(np.uint16).reshape(-1)
for i in range(3):
    tag("decode right after a decode (outputs kept)")
    keep.append(lfm.decode(buf))
for i in range(3):
    tag("after a compare with the reference")
    ok = bool(np.array_equal(keep[-1].reshape(-1), ref))
    keep.append(lfm.decode(buf))
for i in range(3):
    tag("after reading the reference (sum)")
    _ = int(ref[::512].sum())
    keep.append(lfm.decode(buf))
for i in range(3):
    tag("after a compare of two decode outputs")
    ok = bool(np.array_equal(keep[-1], keep[-2]))
    keep.append(lfm.decode(buf))
for i in range(3):
    tag("after freeing an unrelated touched 537 MB array")
    a = np.ones(X * Y * Z, np.uint16)
    del a
    keep.append(lfm.decode(buf))
for i in range(3):
    tag("after freeing an older decode output")
    del keep[0]
    keep.append(lfm.decode(buf))
for i in range(3):
    tag("after freeing the previous decode output")
    del keep[-1]
    keep.append(lfm.decode(buf))
for i in range(3):
    tag("after freeing an unrelated array written from pinned memory")
    a = np.empty(X * Y * Z, np.uint16)
    p = torch.empty(X * Y * Z, dtype=torch.int16).pin_memory()
    a[:] = p.numpy().view(np.uint16)
    del a, p
    keep.append(lfm.decode(buf))
    del keep[0]
