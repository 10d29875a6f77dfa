"""bench.py's standalone predictor roofline (warm / flushed medians of 20
launches plus the same-box copy ceilings) without the rest of the bench, for
A/B of predictor builds (LFM_LIB=variants/<name>/liblfm.so).
usage: python scripts/pred_standalone.py [label]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
import torch  # noqa: E402

torch.cuda.set_device(0)
bench.lfm.require_gpu()
bench.lfm.set_family(bench.FAMILY)
d = torch.empty((bench.Z, bench.Y, bench.X), dtype=torch.int16, device="cuda")
bench.lfm.synth_device(d, bench.X, bench.Y, bench.Z, bench.T, t_index=0, idx0=0, seed=0x4C464D03)
torch.cuda.synchronize()
k, _ = bench.lfm.select_device(d[0], bench.X, bench.Y, bench.T, bench.FAMILY)
alg = 4 * bench.X * bench.Y * bench.Z
r = bench.predictor_standalone(d, bench.Z, int(k), alg)
print(json.dumps({"label": sys.argv[1] if len(sys.argv) > 1 else os.environ.get("LFM_LIB", "base"), **r}))
