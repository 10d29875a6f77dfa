"""Kernel-level timing of the HIP path (HIP events on one stream, inputs resident in HBM).

python scripts/bench_kernels.py [--families tiles,angle,space] [--preds 1-7] [--iters 20]
Prints one JSON line per (kernel, family, predictor) with time and GB/s (algorithmic bytes).
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lightfieldmicroscopy_pc-bzip2_amd"))
import torch  # noqa: E402
import lfm  # noqa: E402


def timeit(fn, iters, stream):
    fn()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(iters):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--X", type=int, default=2048)
    ap.add_argument("--Y", type=int, default=2048)
    ap.add_argument("--Z", type=int, default=64)
    ap.add_argument("--T", type=int, default=15)
    ap.add_argument("--families", default="angle")
    ap.add_argument("--preds", default="1,2,3,4,5,6,7")
    ap.add_argument("--video", type=int, default=0)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--select", type=int, default=1)
    ap.add_argument("--unpredict", type=int, default=1)
    ap.add_argument("--decode", type=int, default=0, help="time whole-file decode of an encoded stack")
    a = ap.parse_args()
    torch.cuda.set_device(0)
    X, Y, Z, T = a.X, a.Y, a.Z, a.T
    d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
    o = torch.empty_like(d)
    lfm.synth_device(d, X, Y, Z, T, seed=0x4C464D03)
    st = torch.cuda.current_stream()
    px = X * Y * Z
    ntemp = (Z // 2) if a.video else 0
    alg = px * 4 + ntemp * X * Y * 2
    for fam in a.families.split(","):
        for k in [int(v) for v in a.preds.split(",")]:
            ms = timeit(lambda: lfm.predict_device(d, o, X, Y, Z, T, fam, k, a.video, stream=st), a.iters, st)
            print(json.dumps({"kernel": "predict", "family": fam, "k": k, "video": a.video, "ms": round(ms, 4),
                              "GBps": round(alg / ms / 1e6, 1), "frac_8TBs": round(alg / ms / 1e6 / 8000, 4)}))
            if a.unpredict and not (a.video and fam != "tiles"):
                lfm.predict_device(d, o, X, Y, Z, T, fam, k, a.video, stream=st)
                r = torch.empty_like(d)
                ms = timeit(lambda: lfm.unpredict_device(o, r, X, Y, Z, T, fam, k, a.video, stream=st),
                            max(3, a.iters // 4), st)
                ok = bool(torch.equal(r, d))
                print(json.dumps({"kernel": "unpredict", "family": fam, "k": k, "video": a.video, "ms": round(ms, 4),
                                  "GBps": round(alg / ms / 1e6, 1), "frac_8TBs": round(alg / ms / 1e6 / 8000, 4),
                                  "exact": ok}))
        if a.decode:
            import time
            lfm.set_family(fam)
            buf, _ = lfm.Encoder(device=0).encode(d, header_version=0, nnum=T)
            lfm.decode(buf)
            t0 = time.perf_counter()
            for _ in range(3):
                out = lfm.decode(buf)
            dt = (time.perf_counter() - t0) / 3
            ok = bool((torch.from_numpy(out.reshape(Z, Y, X).view("int16")) == d.cpu()).all())
            print(json.dumps({"kernel": "decode_file", "family": fam, "s": round(dt, 4),
                              "Mpx_per_s": round(px / dt / 1e6, 1), "bytes": len(buf), "exact": ok}))
        if a.select:
            ms = timeit(lambda: lfm.select_device(d[0], X, Y, T, fam, stream=st), max(3, a.iters // 4), st)
            print(json.dumps({"kernel": "select", "family": fam, "ms": round(ms, 4), "frame": [X, Y]}))


if __name__ == "__main__":
    main()
