"""One GPU-bzip2 batch of config-3 symbols, alone on the device (no second
batch overlapping it): a short program for rocprofv3 kernel traces of the
per-stream stages.  usage: python scripts/bz_probe.py [reps] [streams]"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lightfieldmicroscopy_pc-bzip2_amd"))
import lfm  # noqa: E402

X, Y, Z, T = 2048, 2048, 64, 15
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
count = int(sys.argv[2]) if len(sys.argv) > 2 else 1936
torch.cuda.set_device(0)
lfm.require_gpu()
d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
lfm.synth_device(d, X, Y, Z, T, t_index=0, idx0=0, seed=0x4C464D03)
sym = torch.empty_like(d)
lfm.predict_device(d, sym, X, Y, Z, T, "angle", 4)
torch.cuda.synchronize()
for r in range(reps):
    t0 = time.time()
    out, flags = lfm.bzip2_device(sym, [X, Y, Z, 1, 1], [96, 96, 8, 1, 1], 2, count=count)
    torch.cuda.synchronize()
    print("rep %d: %.2f ms wall (incl. workspace alloc + D2H), %d host-flagged, %d bytes" %
          (r, 1e3 * (time.time() - t0), sum(flags), sum(len(o) for o in out if o)), flush=True)
    st = (ctypes.c_float * 5)()
    if lfm.lib().lfm_hip_bzip2_last_stage_ms(st) == 0:
        print("  stages ms: rle1 %.3f bwt %.3f mtf %.3f huffman %.3f emit %.3f" % tuple(st), flush=True)
