"""Config 5 streamed from host memory (bench.py's config5_host leg, small):
N t-volumes of 4096 x 4096 x 32 (video, tiles, Nnum 13, auto) in a pageable
host array -> lfm_encoder_encode_multi (warm call timed, stage times
printed) -> per-volume lfm.decode_roi into one reused buffer (times printed).
usage: [LFM_DECODE_TIMING=1] python scripts/c5host_probe.py [nvol] [pinned]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lightfieldmicroscopy_pc-bzip2_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import lfm  # noqa: E402

X, Y, Z, T, seed = 4096, 4096, 32, 13, 0x4C464D05
nvol = int(sys.argv[1]) if len(sys.argv) > 1 else 4
pinned = len(sys.argv) > 2 and sys.argv[2] == "pinned"
torch.cuda.set_device(0)
if pinned:
    ht = torch.empty((nvol, 1, Z, Y, X), dtype=torch.int16, pin_memory=True)
    img = ht.numpy().view(np.uint16)
else:
    img = np.empty((nvol, 1, Z, Y, X), dtype=np.uint16)
d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
for t in range(nvol):
    lfm.synth_device(d, X, Y, Z, T, t_index=t, idx0=t * Z * X * Y, seed=seed)
    torch.from_numpy(img[t, 0].view(np.int16)).copy_(d)
torch.cuda.synchronize()
lfm.set_family("tiles")
lfm.set_devices([0])
enc = lfm.Encoder(device=0)
enc.encode_multi(img[:1], header_version=0x80, nnum=T, copy=True)
out = {"nvol": nvol, "pinned": pinned, "runs": []}
for rep in range(2):
    t0 = time.perf_counter()
    b, st = enc.encode_multi(img, header_version=0x80, nnum=T, copy=False)
    ms = (time.perf_counter() - t0) * 1e3
    out["runs"].append({"ms": round(ms, 1), "Mpixel_per_s": round(nvol * X * Y * Z / ms / 1e3, 1),
                        **{k: round(v, 2) for k, v in st.items() if isinstance(v, float)}})
b = bytes(b)
enc.close()
buf = np.empty((Z, Y, X), dtype=np.uint16)
dec = []
for t in range(nvol):
    t1 = time.perf_counter()
    lfm.decode_roi(b, [0, 0, 0, 0, t], [X - 1, Y - 1, Z - 1, 0, t], out=buf)
    dec.append(round((time.perf_counter() - t1) * 1e3, 1))
out["decode_roi_ms"] = dec
print(json.dumps(out), flush=True)
