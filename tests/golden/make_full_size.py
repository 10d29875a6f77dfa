"""Full-size oracle digests for the BASELINE configs (SURVEY.md section 7 step 1:
"SHA-256 of the .lfm for the large configs").

TEST INFRASTRUCTURE.  Run in the build container after `make -C oracle` (so the
reference's own bzip2-1.0.6 is in oracle/_ref):
    python tests/golden/make_full_size.py [--only NAME] [--threads N]

Each stack is generated slab by slab (one block depth of frames at a time) by
the SURVEY 8(d) generator, predicted by the oracle's C restatement (selection
on frame 0, klb_imageIO.cpp:2316-2360; temporal frames `video & z` with the
previous raw frame, :1244-1313), split into the reference's x-fastest blocks
(:98-160) and compressed by BZ2_bzBuffToBuffCompress(level, 0, 30) of the
reference's vendored bzip2-1.0.6 (:217) on a thread pool; the header and the
cumulative end-offset table (:1145-1225) are then hashed with the payload.
Writes tests/golden/full_size_manifest.json: SHA-256 and size of every .lfm,
the chosen predictor, and a SHA-256 per layer of blocks (one block depth of
frames) so a mismatch on the GPU names the layer.
"""
import argparse
import hashlib
import json
import math
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import lfm_oracle as O  # noqa: E402

# name: (X, Y, Z, T, family, header_version, seed); c = t = 1 for every entry
CONFIGS = {
    # config 3: the roofline / bench config (bench.py hashes its .lfm against this)
    "cfg3_2048x2048x64_angle_auto": (2048, 2048, 64, 15, "angle", 0x00, 0x4C464D03),
    # config 3 weak-scaled to 8 GPUs (bench.py --gpus N: rank r encodes frames
    # 64r .. 64r+63 of this stack); its per-layer digests check the merged file
    "cfg3x8_2048x2048x512_angle_auto": (2048, 2048, 512, 15, "angle", 0x00, 0x4C464D03),
    # config 4: entropy-selected predictor (tiles), the 8-GPU z-slab config
    "cfg4_2048x2048x256_tiles_auto": (2048, 2048, 256, 15, "tiles", 0x00, 0x4C464D04),
    # config 5: one t-volume (t = 0) of the 4096 x 4096 x 32 x 1 x 100 video stack;
    # blocks never span t, so every t-volume is coded alone
    "cfg5v0_4096x4096x32_video_tiles_auto": (4096, 4096, 32, 13, "tiles", 0x80, 0x4C464D05),
    # config 5, four t-volumes (t = 0..3) of the same stack: one .lfm of the
    # 4096 x 4096 x 32 x 1 x 4 video stack; selection on frame 0 of volume 0,
    # every volume's z loop coded alone;
    # volume_sha256[t] = SHA-256 of volume t's block streams
    "cfg5x4_4096x4096x32x1x4_video_tiles_auto": (4096, 4096, 32, 13, "tiles", 0x80, 0x4C464D05, 4),
}
# config 5, far t-volumes of the 100-volume stack (4096 x 4096 x 32 x 1 x 100):
# volume_sha256[t] for t in FAR_VOLUMES, each volume's block streams coded
# alone with the predictor chosen on volume 0's frame 0.  In the 100-volume
# .lfm (51.6 GB) these streams sit at end-offsets far past 2^32, so checking
# them checks the u64 offset table (klb_imageHeader.h:46) as well.
FAR_NAME = "cfg5far_4096x4096x32x1x100_video_tiles_auto"
FAR_VOLUMES = (50, 99)
BLOCK = [96, 96, 8, 1, 1]  # default uint16 block (klb_imageHeader.cpp:301-309)


def volume_digests(X, Y, Z, T, family, hv, seed, threads, ts):
    """SHA-256 and byte count of the block streams of t-volumes `ts` of the
    video stack (volume t alone, predictor chosen on volume 0's frame 0)."""
    bz = O.bzip2()
    assert "reference" in bz.kind, "build oracle/_ref first (make -C oracle)"
    video = hv >> 7
    f0 = O.synthetic_lf(X, Y, Z=1, T=T, seed=seed)[0, 0, 0]
    k, _ = O.select(f0, T, family)
    bs = [min(b, x) for b, x in zip(BLOCK, [X, Y, Z, 1, 1])]
    level = min(9, -(-2 * int(np.prod(bs)) // 100000))
    nbx, nby = math.ceil(X / bs[0]), math.ceil(Y / bs[1])
    out = {}
    with ThreadPoolExecutor(threads) as ex:
        for t in ts:
            h, n, prev_raw = hashlib.sha256(), 0, None
            for z0 in range(0, Z, bs[2]):
                dz = min(bs[2], Z - z0)
                raw = O.synthetic_lf(X, Y, Z=dz, T=T, seed=seed, z0=z0, t0=t, idx0=(t * Z + z0) * X * Y)[0, 0]
                sym = np.empty_like(raw)
                for j in range(dz):
                    z = z0 + j
                    zf = (video & z) & 1
                    p = raw[j - 1] if j else prev_raw
                    sym[j] = O.predict_frame(raw[j], p if zf else None, T, family, k, zf) if k else raw[j]
                prev_raw = raw[-1].copy()

                def one(b):
                    by, bx = divmod(b, nbx)
                    blk = np.ascontiguousarray(sym[:, by * bs[1]:(by + 1) * bs[1], bx * bs[0]:(bx + 1) * bs[0]])
                    return bz.compress(blk.tobytes(), level)
                for blob in ex.map(one, range(nbx * nby)):
                    h.update(blob)
                    n += len(blob)
            out[str(t)] = dict(sha256=h.hexdigest(), bytes=n)
    return dict(chosen=int(k), final_header_version=(hv & 0x80) | int(k), level=level,
                nblocks_per_volume=nbx * nby * math.ceil(Z / bs[2]), volumes=out)


def encode_full(X, Y, Z, T, family, hv, seed, threads, Tn=1):
    bz = O.bzip2()
    assert "reference" in bz.kind, "build oracle/_ref first (make -C oracle)"
    video = hv >> 7
    req = hv & 0x7F
    f0 = O.synthetic_lf(X, Y, Z=1, T=T, seed=seed)[0, 0, 0]
    if req < 8:
        k, ent = O.select(f0, T, family)
    else:
        k, ent = req - 8, None
    hv_out = (hv & 0x80) | k
    bs = [min(b, x) for b, x in zip(BLOCK, [X, Y, Z, 1, Tn])]
    level = min(9, -(-2 * int(np.prod(bs)) // 100000))
    nbx, nby = math.ceil(X / bs[0]), math.ceil(Y / bs[1])
    blobs = []
    layers = []
    volumes = []
    with ThreadPoolExecutor(threads) as ex:
        for t in range(Tn):
            prev_raw = None
            vol = []
            for z0 in range(0, Z, bs[2]):
                dz = min(bs[2], Z - z0)
                raw = O.synthetic_lf(X, Y, Z=dz, T=T, seed=seed, z0=z0, t0=t,
                                     idx0=(t * Z + z0) * X * Y)[0, 0]
                sym = np.empty_like(raw)
                for j in range(dz):
                    z = z0 + j
                    zf = (video & z) & 1
                    p = raw[j - 1] if j else prev_raw
                    sym[j] = O.predict_frame(raw[j], p if zf else None, T, family, k, zf) if k else raw[j]
                prev_raw = raw[-1].copy()

                def one(b):
                    by, bx = divmod(b, nbx)
                    blk = np.ascontiguousarray(sym[:, by * bs[1]:(by + 1) * bs[1], bx * bs[0]:(bx + 1) * bs[0]])
                    return bz.compress(blk.tobytes(), level)
                lay = list(ex.map(one, range(nbx * nby)))
                layers.append(hashlib.sha256(b"".join(lay)).hexdigest())
                vol.extend(lay)
            volumes.append(hashlib.sha256(b"".join(vol)).hexdigest())
            blobs.extend(vol)
    offsets = np.cumsum([len(b) for b in blobs]).astype(np.uint64)
    head = O.header_bytes(hv_out, T, [X, Y, Z, 1, Tn], [1.0] * 5, 1, 1, None, bs, offsets)
    h = hashlib.sha256(head)
    for b in blobs:
        h.update(b)
    size = len(head) + int(offsets[-1])
    return dict(sha256=h.hexdigest(), size=size, final_header_version=hv_out, chosen=int(k),
                entropy=None if ent is None else [float(e) for e in ent], layer_sha256=layers,
                header_sha256=hashlib.sha256(head).hexdigest(), nblocks=len(blobs), level=level,
                ratio=round(X * Y * Z * Tn * 2 / size, 4), **({"volume_sha256": volumes} if Tn > 1 else {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    args = ap.parse_args()
    path = os.path.join(HERE, "full_size_manifest.json")
    man = {e["name"]: e for e in json.load(open(path))} if os.path.exists(path) else {}
    for name, cfg in CONFIGS.items():
        X, Y, Z, T, fam, hv, seed = cfg[:7]
        Tn = cfg[7] if len(cfg) > 7 else 1
        if args.only and args.only != name:
            continue
        t0 = time.time()
        r = encode_full(X, Y, Z, T, fam, hv, seed, args.threads, Tn)
        gen = "synthetic_lf(%d,%d,%d,T=%d,seed=0x%X)" % (X, Y, Z, T, seed)
        if Tn > 1:
            gen = "synthetic_lf(%d,%d,%d,Tn=%d,T=%d,seed=0x%X), one volume at a time (t0, idx0)" % (X, Y, Z, Tn, T,
                                                                                                  seed)
        e = dict(name=name, xyzct=[X, Y, Z, 1, Tn], nnum=T, family=fam, header_version=hv, seed=seed,
                 block_size=BLOCK, generator=gen, bzip2=O.bzip2().kind, **r)
        man[name] = e
        print("%s: %d bytes, predictor %d, ratio %.3f, %.1f s" % (name, e["size"], e["chosen"], e["ratio"],
                                                                  time.time() - t0), flush=True)
    if not args.only or args.only == FAR_NAME:
        t0 = time.time()
        X, Y, Z, T, fam, hv, seed = 4096, 4096, 32, 13, "tiles", 0x80, 0x4C464D05
        r = volume_digests(X, Y, Z, T, fam, hv, seed, args.threads, FAR_VOLUMES)
        man[FAR_NAME] = dict(name=FAR_NAME, xyzct=[X, Y, Z, 1, 100], nnum=T, family=fam, header_version=hv,
                             seed=seed, block_size=BLOCK, bzip2=O.bzip2().kind,
                             generator="synthetic_lf(%d,%d,%d,T=%d,seed=0x%X, t0=t, idx0=t*Z*X*Y) per volume"
                             % (X, Y, Z, T, seed), **r)
        print("%s: volumes %s, %.1f s" % (FAR_NAME, list(FAR_VOLUMES), time.time() - t0), flush=True)
    with open(path, "w") as f:
        json.dump(list(man.values()), f, indent=1)


if __name__ == "__main__":
    main()
