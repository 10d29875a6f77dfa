"""Median wall time of one 2048^2 predictor selection (lfm_hip_select: seven
candidates, 2D entropies, argmin; synchronous) on the bench's frame 0.
usage: python scripts/select_probe.py [label]   (LFM_LIB selects a build)"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lightfieldmicroscopy_pc-bzip2_amd"))
import lfm  # noqa: E402

X, Y, T = 2048, 2048, 15
torch.cuda.set_device(0)
lfm.require_gpu()
d = torch.empty((1, Y, X), dtype=torch.int16, device="cuda")
lfm.synth_device(d, X, Y, 1, T, t_index=0, idx0=0, seed=0x4C464D03)
torch.cuda.synchronize()
ts = []
for i in range(25):
    t0 = time.perf_counter()
    k, ent = lfm.select_device(d[0], X, Y, T, "angle")
    ts.append((time.perf_counter() - t0) * 1e3)
print(json.dumps({"label": sys.argv[1] if len(sys.argv) > 1 else "base", "chosen": int(k),
                  "select_ms_median": round(float(np.median(ts[5:])), 3), "select_ms_min": round(min(ts[5:]), 3)}))
