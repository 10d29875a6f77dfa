"""Generates the committed golden fixtures under tests/golden/ from the CPU oracle.

Run from the repo root after `make -C oracle`:
    python tests/golden/make_golden.py [--reference /root/reference]

Outputs (all small):
  predictor_vectors.npz  inputs + expected symbols for every family x predictor
                         x {spatial, temporal} on edge shapes (W, H not multiples
                         of Nnum, Nnum in {1,2,5,13,15,31,40}, tiny frames, full-range
                         uint16 noise that exercises the int16 wrap)
  entropy_vectors.json   candidate entropies + selected predictor for seeded frames
  lfm_manifest.json      oracle .lfm SHA-256 / size for the BASELINE configs at
                         sizes the oracle finishes quickly, plus small .lfm files
  lfm_small/*.lfm        the small .lfm files themselves
  img_tif.npz            testData/img.tif (29 x 151 x 101 uint16, the reference's
                         own test input), copied as data when --reference exists
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import lfm_oracle as O  # noqa: E402

FAMS = ["tiles", "angle", "space"]
# (W, H, T, kind)
SHAPES = [(16, 16, 4, "lf"), (45, 31, 13, "lf"), (64, 48, 15, "lf"), (40, 40, 5, "noise"), (1, 1, 13, "noise"),
          (13, 13, 13, "lf"), (14, 14, 13, "noise"), (33, 7, 2, "noise"), (9, 11, 1, "noise"),
          (96, 70, 31, "lf"), (120, 90, 40, "noise"), (520, 40, 15, "lf"), (1032, 20, 13, "noise")]


def frames_for(W, H, T, kind, seed):
    if kind == "lf":
        a = O.synthetic_lf(W, H, Z=2, T=T, seed=seed)[0, 0]
    else:
        rng = np.random.default_rng(seed)
        a = rng.integers(0, 65536, size=(2, H, W), dtype=np.uint16)
    return np.ascontiguousarray(a)


def predictor_vectors():
    out = {}
    for si, (W, H, T, kind) in enumerate(SHAPES):
        tag = "s%d_%dx%d_T%d" % (si, W, H, T)
        fr = frames_for(W, H, T, kind, 0x4C464D00 + si)
        out["in_" + tag] = fr
        for fam in FAMS:
            for k in range(1, 8):
                out["%s_%s_k%d_z0" % (tag, fam, k)] = O.predict_frame(fr[1], None, T, fam, k, 0)
                out["%s_%s_k%d_z1" % (tag, fam, k)] = O.predict_frame(fr[1], fr[0], T, fam, k, 1)
    np.savez_compressed(os.path.join(HERE, "predictor_vectors.npz"), **out)
    return len(out)


def entropy_vectors():
    rows = []
    cases = [(64, 64, 13, "lf"), (512, 512, 13, "lf"), (97, 53, 15, "noise"), (300, 1600, 15, "lf"),
             (128, 128, 13, "zeros")]
    for i, (W, H, T, kind) in enumerate(cases):
        if kind == "zeros":
            fr = np.zeros((H, W), dtype=np.uint16)
        else:
            fr = frames_for(W, H, T, kind, 0x4C464D10 + i)[1]
        for fam in FAMS:
            k, ent = O.select(fr, T, fam)
            rows.append(dict(W=W, H=H, T=T, kind=kind, seed=0x4C464D10 + i, family=fam, chosen=int(k),
                             entropy=[float(e) for e in ent]))
    with open(os.path.join(HERE, "entropy_vectors.json"), "w") as f:
        json.dump(rows, f, indent=1)
    return len(rows)


def sha(b):
    return hashlib.sha256(b).hexdigest()


def lfm_manifest(img_tif):
    os.makedirs(os.path.join(HERE, "lfm_small"), exist_ok=True)
    entries = []

    def add(name, img, hv, nnum, fam, block=None, keep=False, gen=None):
        b = O.encode(img, header_version=hv, nnum=nnum, family=fam, block_size=block)
        e = dict(name=name, header_version=hv, nnum=nnum, family=fam, block_size=block, sha256=sha(b), size=len(b),
                 final_header_version=b[0], shape_tczyx=list(np.asarray(img).shape), generator=gen)
        if keep:
            with open(os.path.join(HERE, "lfm_small", name + ".lfm"), "wb") as f:
                f.write(b)
            e["file"] = "lfm_small/%s.lfm" % name
        entries.append(e)

    if img_tif is not None:
        # config 1: img.tif page 0 (all zeros), predictor off (request 8), default blocks
        add("cfg1_imgtif_page0_req8", img_tif[0][None, None, None], 8, 13, "tiles", keep=True, gen="img_tif[0]")
        add("cfg1_imgtif_stack_req8", img_tif[None, None], 8, 13, "tiles", keep=True, gen="img_tif")
        add("imgtif_page12_auto", img_tif[12][None, None, None], 0, 13, "tiles", keep=True, gen="img_tif[12]")
        add("imgtif_stack_auto_video", img_tif[None, None], 0x80, 13, "tiles", keep=True, gen="img_tif")
        add("matlab_test_m", img_tif[0][None, None, None], 7, 13, "tiles", block=[101, 151, 1, 1, 1], keep=True,
            gen="img_tif[0]")
    # config 2: 512 x 512, Nnum 13, space family, auto-select (exact BASELINE size)
    g2 = O.synthetic_lf(512, 512, Z=1, T=13, seed=0x4C464D02)
    add("cfg2_512x512_space_auto", g2, 0, 13, "space", gen="synthetic_lf(512,512,1,T=13,seed=0x4C464D02)")
    # config 3 scaled: 512 x 512 x 8, Nnum 15, angle, auto on frame 0
    g3 = O.synthetic_lf(512, 512, Z=8, T=15, seed=0x4C464D03)
    add("cfg3s_512x512x8_angle_auto", g3, 0, 15, "angle", gen="synthetic_lf(512,512,8,T=15,seed=0x4C464D03)")
    # config 4 scaled: 256 x 256 x 16 tiles auto
    g4 = O.synthetic_lf(256, 256, Z=16, T=15, seed=0x4C464D04)
    add("cfg4s_256x256x16_tiles_auto", g4, 0, 15, "tiles", gen="synthetic_lf(256,256,16,T=15,seed=0x4C464D04)")
    # config 5 scaled: 128 x 128 x 8 x 1 x 3 video, tiles, forced predictor of volume 0's choice
    g5 = O.synthetic_lf(128, 128, Z=8, C=1, Tn=3, T=13, seed=0x4C464D05)
    add("cfg5s_128x128x8x1x3_video_auto", g5, 0x80, 13, "tiles",
        gen="synthetic_lf(128,128,8,1,3,T=13,seed=0x4C464D05)")
    # config 5 scaled as SURVEY 8(d) states it: 512 x 512 x 32 x 1 x 3 video, tiles, auto
    g5b = O.synthetic_lf(512, 512, Z=32, C=1, Tn=3, T=13, seed=0x4C464D05)
    add("cfg5s_512x512x32x1x3_video_auto", g5b, 0x80, 13, "tiles",
        gen="synthetic_lf(512,512,32,1,3,T=13,seed=0x4C464D05)")
    small = O.synthetic_lf(70, 45, Z=3, T=13, seed=0x4C464D06)
    for fam in FAMS:
        for k in range(8):
            add("small_%s_req%d" % (fam, 8 + k), small, 8 + k, 13, fam, block=[32, 16, 2, 1, 1], keep=True,
                gen="synthetic_lf(70,45,3,T=13,seed=0x4C464D06)")
    with open(os.path.join(HERE, "lfm_manifest.json"), "w") as f:
        json.dump(entries, f, indent=1)
    return len(entries)


def load_img_tif(ref):
    p = os.path.join(ref, "testData", "img.tif")
    if not os.path.exists(p):
        return None
    from PIL import Image
    im = Image.open(p)
    pages = []
    for i in range(im.n_frames):
        im.seek(i)
        pages.append(np.array(im, dtype=np.uint16))
    a = np.stack(pages)
    np.savez_compressed(os.path.join(HERE, "img_tif.npz"), img=a)
    return a


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    img = load_img_tif(args.reference)
    if img is None and os.path.exists(os.path.join(HERE, "img_tif.npz")):
        img = np.load(os.path.join(HERE, "img_tif.npz"))["img"]
    print("predictor vectors:", predictor_vectors())
    print("entropy vectors:", entropy_vectors())
    print("lfm manifest entries:", lfm_manifest(img))
