import os, sys, json, bz2
import numpy as np
sys.path.insert(0, "lightfieldmicroscopy_pc-bzip2_amd"); sys.path.insert(0, "oracle")
import torch, lfm
import lfm_oracle as O
X, Y, Z, T = 2048, 2048, 64, 15
d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
lfm.synth_device(d, X, Y, Z, T, seed=0x4C464D03)
lfm.set_family("space")
buf, st = lfm.Encoder(device=0).encode(d, header_version=0, nnum=T)
buf = bytes(buf)
h = O.parse_header(buf)
k = h["header_version"] & 0x7F
sym = torch.empty_like(d)
lfm.predict_device(d, sym, X, Y, Z, T, "space", k, 0)
symh = sym.cpu().numpy().view(np.uint16)
bad = []
prev = 0
os.makedirs("gpurun_out", exist_ok=True)
for bid, coord, size in O.iter_blocks(h["xyzct"], h["block_size"]):
    end = int(h["offsets"][bid]); blob = buf[h["header_size"] + prev: h["header_size"] + end]; prev = end
    x0, y0, z0, _, _ = coord; sx, sy, sz, _, _ = size
    raw = np.ascontiguousarray(symh[z0:z0 + sz, y0:y0 + sy, x0:x0 + sx]).tobytes()
    ok = True
    try:
        ok = bz2.decompress(blob) == raw
    except Exception:
        ok = False
    if not ok:
        if not bad:
            open("gpurun_out/bad_raw.bin", "wb").write(raw)
            open("gpurun_out/bad_gpu.bz2", "wb").write(blob)
        bad.append(bid)
print(json.dumps({"hv": h["header_version"], "bs": h["block_size"], "nb": h["nb"], "bad": bad[:20], "nbad": len(bad)}))
