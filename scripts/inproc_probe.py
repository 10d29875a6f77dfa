"""Drop-in writer from host memory (bench.py's inproc leg, config 4:
2048 x 2048 x 256 uint16, tiles, Nnum 15, auto) on one device: per-call
stage times of lfm_encoder_encode_multi (h2d = the uploader's wall time,
compress = GPU bzip2 + assembly), for the environment it runs under.
usage: python scripts/inproc_probe.py [reps]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lightfieldmicroscopy_pc-bzip2_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lfm  # noqa: E402

X, Y, Z, T = 2048, 2048, 256, 15
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
torch.cuda.set_device(0)
d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
lfm.synth_device(d, X, Y, Z, T, seed=0x4C464D04)
host = torch.empty((Z, Y, X), dtype=torch.int16, pin_memory=True)
host.copy_(d)
del d
arr = host.numpy().view(np.uint16)
lfm.set_family("tiles")
lfm.set_devices([0])
enc = lfm.Encoder(device=0)
runs = []
for i in range(reps + 1):
    t0 = time.perf_counter()
    b, st = enc.encode_multi(arr, header_version=0, nnum=T, copy=False)
    ms = (time.perf_counter() - t0) * 1e3
    if i:
        runs.append({"ms": round(ms, 2), "Mpixel_per_s": round(X * Y * Z / ms / 1e3, 1),
                     **{k: round(st[k], 2) for k in ("h2d_ms", "select_ms", "predict_ms", "compress_ms", "d2h_ms")}})
enc.close()
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("LFM_")}, "runs": runs}), flush=True)
