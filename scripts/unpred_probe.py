"""Inverse-predictor timing by shape (decode critical path): one band, one
frame, the config-3 stack; LFM_UNPREDICT_XCU selects band5 (default) / band4.
python scripts/unpred_probe.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lightfieldmicroscopy_pc-bzip2_amd"))
import torch  # noqa: E402
import lfm  # noqa: E402

torch.cuda.set_device(0)
st = torch.cuda.current_stream()
for (X, Y, Z) in [(2048, 64, 1), (2048, 128, 1), (2048, 512, 1), (2048, 2048, 1), (2048, 2048, 8), (2048, 2048, 64)]:
    T = 15
    d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
    lfm.synth_device(d, X, Y, Z, T, seed=0x4C464D03)
    s = torch.empty_like(d)
    r = torch.empty_like(d)
    lfm.predict_device(d, s, X, Y, Z, T, "angle", 4, 0, stream=st)
    lfm.unpredict_device(s, r, X, Y, Z, T, "angle", 4, 0, stream=st)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    n = 5
    for _ in range(n):
        lfm.unpredict_device(s, r, X, Y, Z, T, "angle", 4, 0, stream=st)
    e1.record(st)
    torch.cuda.synchronize()
    print(json.dumps({"shape": [X, Y, Z], "ms": round(e0.elapsed_time(e1) / n, 4), "exact": bool(torch.equal(r, d)),
                      "xcu": os.environ.get("LFM_UNPREDICT_XCU", "1")}), flush=True)
