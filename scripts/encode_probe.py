"""Config 3 encode from HBM, a few times (the bench's workload without its
legs): a short program to run under rocprofv3 --pmc passes for the fused
predictor kernel (predict_vec<1,4,15,...>, angle family, predictor 4).
usage: python scripts/encode_probe.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lightfieldmicroscopy_pc-bzip2_amd"))
import lfm  # noqa: E402

X, Y, Z, T = 2048, 2048, 64, 15
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
torch.cuda.set_device(0)
lfm.require_gpu()
lfm.set_family("angle")
d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
lfm.synth_device(d, X, Y, Z, T, t_index=0, idx0=0, seed=0x4C464D03)
torch.cuda.synchronize()
enc = lfm.Encoder(device=0, num_threads=16)
for _ in range(reps):
    enc.encode_slab(d, 0, header_version=0, nnum=T, copy=False)
enc.close()
print("ok", flush=True)
