"""Band hand-over trace of the inverse predictor (band5): per band, start,
end and time spent in the per-round waits, from the 100 MHz timestamps the
kernel records under LFM_UNPREDICT_TRACE.
python scripts/unpred_trace.py [OUTDIR]"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "utrace")
os.makedirs(OUT, exist_ok=True)
TRACE = os.path.join(OUT, "trace.bin")
os.environ["LFM_UNPREDICT_TRACE"] = TRACE
sys.path.insert(0, os.path.join(REPO, "lightfieldmicroscopy_pc-bzip2_amd"))
import torch  # noqa: E402
import lfm  # noqa: E402


def read_traces(path):
    raw = open(path, "rb").read()
    off, out = 0, []
    while off < len(raw):
        nfr, nb, slots = np.frombuffer(raw, np.int32, 3, off)
        off += 12
        n = int(nfr) * int(nb) * int(slots)
        t = np.frombuffer(raw, np.uint64, n, off).reshape(int(nb), int(nfr), int(slots)).astype(np.int64)
        off += 8 * n
        out.append(t)
    return out


torch.cuda.set_device(0)
st = torch.cuda.current_stream()
for (X, Y, Z) in [(2048, 128, 1), (2048, 512, 1), (2048, 2048, 1), (2048, 2048, 64)]:
    T = 15
    d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
    lfm.synth_device(d, X, Y, Z, T, seed=0x4C464D03)
    s = torch.empty_like(d)
    r = torch.empty_like(d)
    lfm.predict_device(d, s, X, Y, Z, T, "angle", 4, 0, stream=st)
    for rep in range(2):
        if os.path.exists(TRACE):
            os.remove(TRACE)
        lfm.unpredict_device(s, r, X, Y, Z, T, "angle", 4, 0, stream=st)
        torch.cuda.synchronize()
    exact = bool(torch.equal(r, d))
    (t,) = read_traces(TRACE)
    nb, nfr, slots = t.shape
    t0 = t[:, :, 0][t[:, :, 0] > 0].min()
    rows = []
    for b in range(nb):
        f = 0
        ts = t[b, f]
        rounds = [(ts[1 + 2 * i], ts[2 + 2 * i]) for i in range((slots - 2) // 2) if ts[2 + 2 * i] > 0]
        wait = sum(int(a2 - a1) for a1, a2 in rounds)
        rows.append({"band": b, "start_us": (ts[0] - t0) / 100, "end_us": (ts[slots - 1] - t0) / 100,
                     "dur_us": (ts[slots - 1] - ts[0]) / 100, "wait_us": wait / 100, "rounds": len(rounds),
                     "first_wait_us": (int(rounds[0][1] - rounds[0][0]) / 100) if rounds else 0})
    tot = (t[:, :, slots - 1].max() - t0) / 100
    print(json.dumps({"shape": [X, Y, Z], "exact": exact, "span_us": float(tot),
                      "bands": [{k: round(float(v), 1) for k, v in row.items()} for row in rows[:6]] +
                               ([{k: round(float(v), 1) for k, v in rows[-1].items()}] if nb > 6 else [])}),
          flush=True)
    # every frame's last band end, for the many-frame shape
    if nfr > 1:
        ends = (t[nb - 1, :, slots - 1] - t0) / 100
        starts = (t[0, :, 0] - t0) / 100
        print(json.dumps({"frames": int(nfr), "frame_start_us_min_max": [float(starts.min()), float(starts.max())],
                          "frame_end_us_min_max": [float(ends.min()), float(ends.max())]}), flush=True)
