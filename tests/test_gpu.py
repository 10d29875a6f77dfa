"""GPU parity tests: the HIP path (through the C ABI) against the oracle and
the committed golden fixtures.  Bit-exact for symbols, headers and .lfm bytes;
entropies within 1e-5 relative (float summation order is unpinned in the
reference: thrust::reduce)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu
FAMS = ["tiles", "angle", "space"]


def ref_bz2(oracle, data, level):
    """BZ2_bzBuffToBuffCompress(level, 0, 30) of the reference's own
    bzip2-1.0.6, compiled from /root/reference by oracle/Makefile into
    oracle/_ref/libbz2_ref.so (which travels to the GPU box)."""
    bz = oracle.bzip2()
    assert "reference" in bz.kind, "oracle/_ref/libbz2_ref.so missing: run make -C oracle"
    return bz.compress(bytes(data), level)


def dev16(torch, a):
    t = torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).cuda()
    return t


def host16(t):
    return t.cpu().numpy().view(np.uint16)


def run_predict(lfmlib, torch, frames, T, fam, k, video, z0=0, prev=None):
    Z, H, W = frames.shape
    d_in = dev16(torch, frames)
    d_out = torch.empty_like(d_in)
    d_prev = dev16(torch, prev) if prev is not None else None
    lfmlib.predict_device(d_in, d_out, W, H, Z, T, fam, k, video, z0, d_prev)
    torch.cuda.synchronize()
    return host16(d_out)


def test_golden_predictor_vectors(lfmlib, gpu):
    torch = gpu
    g = np.load(os.path.join(GOLDEN, "predictor_vectors.npz"))
    n = 0
    for key in g.files:
        if not key.startswith("in_"):
            continue
        tag = key[3:]
        T = int(tag.split("_T")[1])
        fr = g[key]
        for fam in FAMS:
            for k in range(1, 8):
                sp = run_predict(lfmlib, torch, fr[1:2], T, fam, k, 0)[0]
                assert np.array_equal(sp, g["%s_%s_k%d_z0" % (tag, fam, k)]), (tag, fam, k, "spatial")
                # temporal: frame index 1 of a video stack -> z_flag = 1, prev = frame 0
                tp = run_predict(lfmlib, torch, fr, T, fam, k, 1)[1]
                assert np.array_equal(tp, g["%s_%s_k%d_z1" % (tag, fam, k)]), (tag, fam, k, "temporal")
                n += 2
    assert n > 500


@pytest.mark.parametrize("W,H,T", [(512, 256, 13), (2048, 160, 15), (1032, 200, 15), (520, 300, 31), (64, 64, 2),
                                   (1024, 96, 1), (776, 130, 11)])
def test_fast_kernel_vs_oracle(lfmlib, oracle, gpu, W, H, T):
    """Shapes that take the LDS-ring kernel (W % 8 == 0, T <= 31): several
    strips, partial last strip, several row segments, video stacks."""
    torch = gpu
    stack = oracle.synthetic_lf(W, H, Z=4, T=T, seed=W * 7 + H)[0, 0]
    rng = np.random.default_rng(W + H)
    stack[2] = rng.integers(0, 65536, size=(H, W), dtype=np.uint16)  # full range exercises the int16 wrap
    for fam in FAMS:
        for k in range(1, 8):
            got = run_predict(lfmlib, torch, stack, T, fam, k, 1)
            exp = oracle.predict_volume(stack, T, fam, k, 1)
            assert np.array_equal(got, exp), (fam, k)


@pytest.mark.parametrize("W,H,T,Z", [(2048, 300, 15, 3), (496, 64, 13, 2), (504, 100, 15, 2), (992, 250, 13, 3),
                                      (1000, 34, 15, 1), (520, 700, 13, 1), (32, 40, 15, 2), (4096, 64, 13, 1)])
def test_spatial_stack_shapes_vs_oracle(lfmlib, oracle, gpu, W, H, T, Z):
    """Spatial stacks (no video bit, predict_vec): widths at and around strip
    seams (one strip, a partial last strip, many strips), heights from one
    lens row plus one to many row pieces, every family and predictor, one
    full-range frame for the int16 wrap.  (Written for the round-6
    register-window kernel, which was exact but slower and was dropped.)"""
    torch = gpu
    stack = oracle.synthetic_lf(W, H, Z=Z, T=T, seed=W * 3 + H + Z)[0, 0]
    stack[-1] = np.random.default_rng(W + H).integers(0, 65536, size=(H, W), dtype=np.uint16)
    for fam in FAMS:
        for k in range(1, 8):
            got = run_predict(lfmlib, torch, stack, T, fam, k, 0)
            exp = oracle.predict_volume(stack, T, fam, k, 0)
            assert np.array_equal(got, exp), (fam, k)


@pytest.mark.parametrize("W,H,T", [(2048, 600, 15), (1032, 200, 13), (520, 300, 31), (45, 31, 13), (64, 40, 2)])
def test_candidates_kernel_vs_oracle(lfmlib, oracle, gpu, W, H, T):
    """The selection pass's one-launch seven-candidate kernel equals the oracle
    for every predictor (fast ring shapes and the generic fallback)."""
    torch = gpu
    fr = oracle.synthetic_lf(W, H, Z=1, T=T, seed=W + 3 * H)[0, 0, 0]
    d_out = torch.empty((7, H, W), dtype=torch.int16, device="cuda")
    for fam in FAMS:
        lfmlib.predict_candidates_device(dev16(torch, fr), d_out, W, H, T, fam)
        torch.cuda.synchronize()
        got = d_out.cpu().numpy().view(np.uint16)
        for k in range(1, 8):
            assert np.array_equal(got[k - 1], oracle.predict_frame(fr, None, T, fam, k, 0)), (fam, k)


def test_predict_z0_offset_and_prev(lfmlib, oracle, gpu):
    """A z-slab starting at an odd z of a video stack takes its previous raw
    frame from d_prev (multi-GPU slabs use this)."""
    torch = gpu
    stack = oracle.synthetic_lf(512, 64, Z=6, T=15)[0, 0]
    full = oracle.predict_volume(stack, 15, "tiles", 4, 1)
    got = run_predict(lfmlib, torch, stack[3:], 15, "tiles", 4, 1, z0=3, prev=stack[2:3])
    assert np.array_equal(got, full[3:])


@pytest.mark.parametrize("W,H,T,Z,z0", [(1032, 200, 15, 5, 0), (520, 160, 13, 2, 1), (2048, 96, 13, 3, 1),
                                        (776, 130, 15, 1, 1), (1024, 90, 13, 6, 2)])
def test_video_frame_pairs_vs_oracle(lfmlib, oracle, gpu, W, H, T, Z, z0):
    """Video volumes code each (spatial, temporal) frame pair in one work item
    (predict_vec_pair: the temporal frame's previous frame comes from the
    spatial frame's ring); a temporal first frame (odd z0, previous frame from
    d_prev) and an unpaired last frame run alone.  Every family and
    predictor, partial last strips, full-range frames for the int16 wrap."""
    torch = gpu
    full = oracle.synthetic_lf(W, H, Z=Z + z0, T=T, seed=W + 5 * Z + z0)[0, 0]
    full[-1] = np.random.default_rng(W).integers(0, 65536, size=(H, W), dtype=np.uint16)
    stack = full[z0:]
    prev = full[z0 - 1:z0] if z0 else None
    for fam in FAMS:
        for k in range(1, 8):
            got = run_predict(lfmlib, torch, stack, T, fam, k, 1, z0=z0, prev=prev)
            exp = oracle.predict_volume(full, T, fam, k, 1)[z0:]
            assert np.array_equal(got, exp), (fam, k)


def test_predictor0_is_copy(lfmlib, oracle, gpu):
    torch = gpu
    stack = oracle.synthetic_lf(96, 40, Z=2, T=13)[0, 0]
    assert np.array_equal(run_predict(lfmlib, torch, stack, 13, "tiles", 0, 1), stack)


def test_entropy_and_selection_vs_golden(lfmlib, oracle, gpu):
    torch = gpu
    rows = json.load(open(os.path.join(GOLDEN, "entropy_vectors.json")))
    for r in rows:
        if r["kind"] == "zeros":
            fr = np.zeros((r["H"], r["W"]), np.uint16)
        elif r["kind"] == "lf":
            fr = oracle.synthetic_lf(r["W"], r["H"], Z=2, T=r["T"], seed=r["seed"])[0, 0, 1]
        else:
            fr = np.random.default_rng(r["seed"]).integers(0, 65536, size=(2, r["H"], r["W"]), dtype=np.uint16)[1]
        k, ent = lfmlib.select_device(dev16(torch, fr), r["W"], r["H"], r["T"], r["family"])
        np.testing.assert_allclose(ent, r["entropy"], rtol=1e-5, atol=1e-6)
        srt = sorted(r["entropy"])
        if r["kind"] == "zeros" or srt[1] - srt[0] > 1e-4 * abs(srt[0]):
            assert k == r["chosen"], r


def test_entropy_single_candidate(lfmlib, oracle, gpu):
    torch = gpu
    rng = np.random.default_rng(11)
    for n in (1, 7, 449999, 450000, 450001, 1000003):
        cand = rng.integers(0, 300, size=n, dtype=np.uint16)
        e = lfmlib.entropy_device(dev16(torch, cand))
        assert abs(e - oracle.entropy2d(cand)) <= 1e-5 * max(1.0, abs(e)), n
    # one bin takes every pair (counts far above 16 bits), and the (0, 0) hot bin
    for v in (0x0101, 0x0000, 0xFFFF, 0x00FF):
        cand = np.full(900001, v, dtype=np.uint16)
        e = lfmlib.entropy_device(dev16(torch, cand))
        assert abs(e - oracle.entropy2d(cand)) <= 1e-5 * max(1.0, abs(e)), hex(v)


@pytest.mark.parametrize("dist", ["small", "bytes", "few", "runs"])
def test_entropy_partner_links(lfmlib, oracle, gpu, dist):
    """The selection never builds the sorted pair array: every position's
    bigram partner is the next occurrence of its byte, linked across the
    64-position windows, the four 4 KiB waves and the 16 KiB segments of
    ent_next, then across keys (sentinel, end of L) by ent_link.  Sizes put
    those seams and the chunk / 16-byte tails in every position; the value
    distributions leave keys absent, make one key hold everything, or make
    long runs."""
    torch = gpu
    rng = np.random.default_rng({"small": 1, "bytes": 2, "few": 3, "runs": 4}[dist])
    for n in (1, 2, 8, 9, 31, 32, 33, 2047, 2048, 2049, 8191, 8192, 8193, 24577, 449999, 450000, 450007):
        if dist == "small":
            cand = np.abs(rng.normal(0, 40, size=n)).astype(np.uint16)
        elif dist == "bytes":
            cand = rng.integers(0, 65536, size=n, dtype=np.uint16)
        elif dist == "few":
            cand = rng.choice(np.array([0x0100, 0x0302, 0x0001], np.uint16), size=n)
        else:
            cand = np.repeat(rng.integers(0, 6, size=n // 50 + 1, dtype=np.uint16), 50)[:n]
        e = lfmlib.entropy_device(dev16(torch, cand))
        assert abs(e - oracle.entropy2d(cand)) <= 1e-5 * max(1.0, abs(e)), (dist, n)


def _manifest():
    return {e["name"]: e for e in json.load(open(os.path.join(GOLDEN, "lfm_manifest.json")))}


def _gen(oracle, e):
    img_tif = np.load(os.path.join(GOLDEN, "img_tif.npz"))["img"]
    if e["generator"].startswith("img_tif"):
        return np.asarray(eval(e["generator"], {"img_tif": img_tif})).reshape(e["shape_tczyx"])
    return eval("O." + e["generator"], {"O": oracle})


@pytest.mark.parametrize("name", ["cfg1_imgtif_page0_req8", "cfg1_imgtif_stack_req8", "cfg2_512x512_space_auto", "cfg3s_512x512x8_angle_auto",
                                  "cfg4s_256x256x16_tiles_auto", "cfg5s_128x128x8x1x3_video_auto",
                                  "cfg5s_512x512x32x1x3_video_auto",
                                  "imgtif_page12_auto", "imgtif_stack_auto_video", "matlab_test_m"])
def test_lfm_bytes_match_oracle_manifest(lfmlib, oracle, gpu, tmp_path, name):
    """Whole encode (GPU selection + predictor + host bzip2) gives the oracle's
    .lfm bytes (SHA-256 committed in tests/golden/lfm_manifest.json)."""
    e = _manifest()[name]
    img = _gen(oracle, e)
    lfmlib.set_family(e["family"])
    try:
        p = tmp_path / "o.lfm"
        lfmlib.write_lfm(p, img, predictor_request=e["header_version"] & 0x7F, nnum=e["nnum"],
                         video=e["header_version"] >> 7, block_size=e["block_size"])
        b = p.read_bytes()
        assert b[0] == e["final_header_version"]
        assert hashlib.sha256(b).hexdigest() == e["sha256"], name
        # device-resident input through the encoder API gives the same bytes
        enc = lfmlib.Encoder()
        t = gpu.from_numpy(np.ascontiguousarray(img).view(np.int16)).cuda()
        b2, st = enc.encode(t, header_version=e["header_version"], nnum=e["nnum"], block_size=e["block_size"])
        assert b2 == b and st["chosen"] == (e["final_header_version"] & 0x7F)
        enc.close()
        if e["family"] == "tiles" or not (e["header_version"] >> 7):
            back, _, _ = lfmlib.read_lfm(p)
            assert np.array_equal(back.reshape(img.shape), img)
    finally:
        lfmlib.set_family("tiles")


@pytest.mark.parametrize("fam", FAMS)
def test_forced_predictors_small_files(lfmlib, oracle, gpu, tmp_path, fam):
    man = _manifest()
    small = oracle.synthetic_lf(70, 45, Z=3, T=13, seed=0x4C464D06)
    lfmlib.set_family(fam)
    try:
        for k in range(8):
            e = man["small_%s_req%d" % (fam, 8 + k)]
            p = tmp_path / ("k%d.lfm" % k)
            lfmlib.write_lfm(p, small, predictor_request=8 + k, nnum=13, block_size=e["block_size"])
            assert p.read_bytes() == open(os.path.join(GOLDEN, e["file"]), "rb").read(), (fam, k)
    finally:
        lfmlib.set_family("tiles")


def test_config3_full_size_properties(lfmlib, oracle, gpu):
    """Config 3 at full size (2048 x 2048 x 64, Nnum 15, angle, auto on frame 0):
    the GPU symbols decode back to the input (angle spatial is lossless), and
    sampled frames equal the oracle bit for bit."""
    torch = gpu
    X, Y, Z, T = 2048, 2048, 64, 15
    d_img = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
    lfmlib.synth_device(d_img, X, Y, Z, T, seed=0x4C464D03)
    k, ent = lfmlib.select_device(d_img[0], X, Y, T, "angle")
    f0 = host16(d_img[0])
    ko, ento = oracle.select(f0, T, "angle")
    np.testing.assert_allclose(ent, ento, rtol=1e-5)
    assert k == ko
    d_sym = torch.empty_like(d_img)
    lfmlib.predict_device(d_img, d_sym, X, Y, Z, T, "angle", k, 0)
    torch.cuda.synchronize()
    for z in (0, 31, 63):
        assert np.array_equal(host16(d_sym[z]), oracle.predict_frame(host16(d_img[z]), None, T, "angle", k, 0)), z


@pytest.mark.parametrize("fam", FAMS)
def test_full_size_encode_decode_roundtrip(lfmlib, oracle, gpu, fam):
    """2048 x 2048 x 64 through the whole GPU writer (selection, predictor,
    bzip2 batches) and back through the reader: every pixel returns, and a
    sample of blocks equals the reference's bzip2 byte for byte."""
    torch = gpu
    X, Y, Z, T = 2048, 2048, 64, 15
    d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
    lfmlib.synth_device(d, X, Y, Z, T, seed=0x4C464D03)
    lfmlib.set_family(fam)
    try:
        buf, _ = lfmlib.Encoder(device=0).encode(d, header_version=0, nnum=T)
        out = lfmlib.decode(bytes(buf))
    finally:
        lfmlib.set_family("tiles")
    img = host16(d)
    assert np.array_equal(out.reshape(Z, Y, X), img), fam
    h = oracle.parse_header(bytes(buf))
    k = h["header_version"] & 0x7F
    sym = oracle.predict_volume(img[:8], T, fam, k, 0) if k else img[:8]
    prev = 0
    for bid, coord, size in oracle.iter_blocks(h["xyzct"], h["block_size"]):
        end = int(h["offsets"][bid])
        if coord[2] == 0 and bid % 17 == 0:
            blob = bytes(buf[h["header_size"] + prev:h["header_size"] + end])
            raw = oracle.gather_block(sym[None, None], coord, size)
            assert blob == ref_bz2(oracle, raw, 2), bid
        prev = end


def test_gpu_bzip2_long_tied_list(lfmlib, oracle, gpu):
    """More than 2^24 rotations tied after the first sort (binary alphabet):
    the tie rounds narrow their text keys so group index + text fit 64 bits."""
    torch = gpu
    rng = np.random.default_rng(5)
    n, m = 140000, 125
    data = rng.integers(0, 2, n * m, dtype=np.uint8)
    d = torch.from_numpy(data).cuda()
    got, flags = lfmlib.bzip2_device(d, [n, m, 1, 1, 1], [n, 1, 1, 1, 1], 1, level=2)
    assert not any(flags)
    for i in range(0, m, 8):
        assert got[i] == ref_bz2(oracle, data[i * n:(i + 1) * n].tobytes(), 2), i


def test_synth_generator_matches_numpy(lfmlib, oracle, gpu):
    torch = gpu
    for (X, Y, Z, T) in ((256, 64, 3, 15), (101, 33, 2, 13)):
        d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
        lfmlib.synth_device(d, X, Y, Z, T, seed=0x4C464D03)
        torch.cuda.synchronize()
        assert np.array_equal(host16(d), oracle.synthetic_lf(X, Y, Z=Z, T=T, seed=0x4C464D03)[0, 0])


@pytest.mark.parametrize("fam,video,on_device", [("tiles", True, True), ("tiles", True, False),
                                                 ("angle", False, True)])
def test_slab_encode_and_merge(lfmlib, oracle, gpu, fam, video, on_device):
    """Multi-GPU sharding on one GPU: z-slabs (odd starts with the previous
    raw frame) encoded with the forced predictor, then joined: identical to
    the oracle's one-piece auto-selected encode."""
    from lfm.shard import forced_request, plan_slabs
    torch = gpu
    Z, bs = 20, [64, 32, 3, 1, 1]  # slabs (0, 9), (9, 9), (18, 2): an odd start
    img = oracle.synthetic_lf(200, 96, Z=Z, T=13, seed=0x4C464D08)
    full = oracle.encode(img, header_version=(0x80 if video else 0), nnum=13, family=fam, block_size=bs)
    lfmlib.set_family(fam)
    try:
        enc = lfmlib.Encoder(device=0)
        k, _ = lfmlib.select_device(dev16(torch, img[0, 0, 0]), 200, 96, 13, fam)
        slabs = []
        for z0, d in plan_slabs(Z, 3, 3):
            slab = img[0, 0, z0:z0 + d]
            prev = img[0, 0, z0 - 1] if z0 else None
            if on_device:
                slab = dev16(torch, slab)
                prev = dev16(torch, prev) if prev is not None else None
            b, st = enc.encode_slab(slab, z0, prev=prev, header_version=forced_request(k, video), nnum=13,
                                    block_size=bs)
            slabs.append(b)
        enc.close()
    finally:
        lfmlib.set_family("tiles")
    assert lfmlib.merge_slabs(slabs) == full


def _bz2_cases():
    rng = np.random.default_rng(7)
    cases = {
        "random": rng.integers(0, 256, 40000, dtype=np.uint8),
        "zeros": np.zeros(30000, np.uint8),
        "one_byte": np.array([65], np.uint8),
        "two_bytes": np.array([1, 2], np.uint8),
        "seven": np.array([3, 3, 3, 3, 3, 3, 9], np.uint8),
        "small_alpha": rng.integers(0, 3, 20000, dtype=np.uint8),
        "few_syms": np.repeat(rng.integers(0, 5, 300, dtype=np.uint8), 7),
        "periodic": np.tile(np.array([7, 9], np.uint8), 5000),
        "periodic_runs": np.tile(np.array([1, 1, 1, 1, 1, 2], np.uint8), 3000),
        # ties longer than the text rounds: the doubling fallback resolves them
        "long_repeat": np.concatenate([np.tile(rng.integers(0, 256, 700, dtype=np.uint8), 12),
                                       np.array([1], np.uint8)]),
        "long_repeat_lowalpha": np.concatenate([np.tile(rng.integers(0, 4, 3000, dtype=np.uint8), 9),
                                                np.array([9, 9], np.uint8)]),
    }
    # runs of equal 8-byte prefixes resolved inside the chunk sort (pairs and
    # triples over a 4-symbol alphabet), at and past its run limit of 32 (a
    # 20-byte motif 32 / 33 times), and past its 64-byte compare limit (a
    # 200-byte block three times): the latter two go to the tie rounds
    cases["alpha4"] = rng.integers(0, 4, 90000, dtype=np.uint8)
    for reps in (32, 33):
        motif = rng.integers(0, 256, 20, dtype=np.uint8)
        cases["motif%d" % reps] = np.concatenate(
            [np.concatenate([motif, rng.integers(0, 256, 50, dtype=np.uint8)]) for _ in range(reps)])
    blk = rng.integers(0, 256, 200, dtype=np.uint8)
    cases["tie_past_compare"] = np.concatenate(
        [np.concatenate([blk, rng.integers(0, 256, 300, dtype=np.uint8)]) for _ in range(3)])
    runs = []
    for L in (1, 2, 3, 4, 5, 254, 255, 256, 259, 510, 511, 1000):
        runs.append(np.full(L, L % 251, np.uint8))
        runs.append(np.array([200], np.uint8))
    cases["run_lengths"] = np.concatenate(runs)
    allb = np.concatenate([np.full(1 + (i % 7), i, np.uint8) for i in range(256)] * 20 + [np.array([5], np.uint8)])
    cases["all_bytes"] = allb  # every byte value in use (not periodic: one extra byte)
    # nMTF >= 2^17: the Huffman tables' weights leave the packed heap's 17 bits
    cases["random_wide"] = rng.integers(0, 256, 160000, dtype=np.uint8)
    # geometric byte distribution: code lengths beyond 17 in the first tree
    # (the weight-halving retry of BZ2_hbMakeCodeLengths)
    geo = np.minimum(rng.geometric(0.5, 140000) - 1, 40).astype(np.uint8)
    cases["geometric"] = geo
    cases["geometric_small"] = geo[:30000].copy()
    # two-stage BWT (bwt_induce): descending runs make chains of A rotations
    # longer than the four carried bytes (the text fallback); bytes in threes
    # (RLE1 keeps them) make A rotations induce into their own bucket, mostly
    # into the same 64-position slice; a long run of 0xFB survives RLE1 as a
    # run of equal bytes, leaving types undecided (the stream is sorted whole);
    # 8-bit text-like data
    desc = []
    while sum(len(d) for d in desc) < 60000:
        a = int(rng.integers(20, 256))
        desc.append(np.arange(a, a - int(rng.integers(3, 20)), -1).astype(np.uint8))
        desc.append(rng.integers(0, 256, int(rng.integers(0, 3)), dtype=np.uint8))
    cases["descending"] = np.concatenate(desc)
    cases["ascending"] = np.concatenate([np.arange(a, min(256, a + 12)) for a in rng.integers(0, 250, 6000)]).astype(np.uint8)
    cases["threes"] = np.repeat(rng.integers(0, 40, 20000, dtype=np.uint8), 3)
    cases["fb_runs"] = np.concatenate([np.full(3000, 0xFB, np.uint8), rng.integers(0, 256, 5000, dtype=np.uint8),
                                       np.full(1300, 0xFB, np.uint8), np.array([1, 0xFB, 2], np.uint8)])
    words = [bytes(rng.integers(97, 123, int(rng.integers(1, 9)), dtype=np.uint8)) for _ in range(400)]
    cases["text"] = np.frombuffer(b" ".join(words[int(i)] for i in rng.integers(0, 400, 12000)), np.uint8).copy()
    return cases


def test_gpu_bzip2_matches_libbz2_edge_cases(lfmlib, oracle, gpu):
    """Every GPU stream equals the reference's bzip2-1.0.6 at the same level;
    periodic blocks come back flagged for the host library."""
    torch = gpu
    for name, data in _bz2_cases().items():
        n = len(data)
        d = torch.from_numpy(data.copy()).cuda()
        for level in (1, 2, 9):
            got, flags = lfmlib.bzip2_device(d, [n, 1, 1, 1, 1], [n, 1, 1, 1, 1], 1, level=level)
            exp = ref_bz2(oracle, data.tobytes(), level)
            if flags[0]:  # periodic, or a second bzip2 block (nblockMAX = 100000 * level - 19)
                assert name.startswith("periodic") or n >= 100000 * level - 19, (name, level)
                continue
            assert not name.startswith("periodic"), name
            assert got[0] == exp, (name, level, len(got[0]), len(exp))


@pytest.mark.parametrize("repeats", [False, True])
def test_gpu_bzip2_mixed_batch(lfmlib, oracle, gpu, repeats):
    """The edge cases as the streams of ONE batch (padded to a common length
    with distinct random tails): induced and whole-sorted streams and host
    fallbacks side by side; with the long repeats, ties that need doubling
    restart the batch with every rotation sorted."""
    torch = gpu
    rng = np.random.default_rng(5)
    slow = ("long_repeat", "tie_past", "motif", "periodic")
    items = [(k, c) for k, c in _bz2_cases().items() if len(c) <= 100000 and (repeats or not k.startswith(slow))]
    names = [k for k, _ in items]
    cases = [c for _, c in items]
    n = max(len(c) for c in cases) + 64
    img = np.stack([np.concatenate([c, rng.integers(0, 256, n - len(c), dtype=np.uint8)]) for c in cases])
    d = torch.from_numpy(img.reshape(-1).copy()).cuda()
    got, flags = lfmlib.bzip2_device(d, [n, 1, len(cases), 1, 1], [n, 1, 1, 1, 1], 1, level=2)
    # the induction cases must run on the device, not fall back to the host
    for name in ("descending", "threes", "text", "ascending"):
        if name in names:
            assert not flags[names.index(name)], name
    checked = 0
    for i in range(len(cases)):
        exp = ref_bz2(oracle, img[i].tobytes(), 2)
        if flags[i]:
            continue
        assert got[i] == exp, names[i]
        checked += 1
    assert checked >= len(cases) - 3, (checked, len(cases), [names[i] for i in range(len(cases)) if flags[i]])


def test_gpu_bzip2_block_grid_and_symbols(lfmlib, oracle, gpu):
    """Many streams from a 2-D block grid of predicted light-field symbols
    (border blocks, uint16 samples) against the reference's bzip2 per block."""
    torch = gpu
    img = oracle.synthetic_lf(200, 150, Z=5, T=13, seed=21)[0, 0]
    sym = oracle.predict_volume(img, 13, "tiles", 4, 0)
    d = torch.from_numpy(sym.view(np.int16).copy()).cuda()
    dims, bs = [200, 150, 5, 1, 1], [64, 48, 2, 1, 1]
    got, flags = lfmlib.bzip2_device(d, dims, bs, 2)
    blocks = list(oracle.iter_blocks(dims, bs))
    assert len(got) == len(blocks)
    for (i, coord, size), g in zip(blocks, got):
        raw = oracle.gather_block(sym[None, None], coord, size)
        assert g == ref_bz2(oracle, raw, 1), i


def test_gpu_bzip2_many_wide_heaps(lfmlib, oracle, gpu):
    """200 random 160 kB streams: 1 200 Huffman tables whose weights leave the
    packed heap's 17 bits, more than one pass of the wide-heap kernel's grid;
    mixed with low-entropy streams (packed heaps) in the same batch."""
    torch = gpu
    rng = np.random.default_rng(11)
    n, ns = 160000, 200
    img = rng.integers(0, 256, (ns, n), dtype=np.uint8)
    img[::7] = rng.integers(0, 4, (len(img[::7]), n), dtype=np.uint8)
    d = torch.from_numpy(img.reshape(-1).copy()).cuda()
    got, flags = lfmlib.bzip2_device(d, [n, 1, ns, 1, 1], [n, 1, 1, 1, 1], 1)
    assert not any(flags)
    for i in range(ns):
        assert got[i] == ref_bz2(oracle, img[i].tobytes(), 2), i


def test_gpu_bzip2_host_fallback_streams(lfmlib, oracle, gpu):
    """A stream whose RLE1 block reaches nblockMAX (runs of exactly four bytes
    expand it by 5/4; libbzip2 would cut a second bzip2 block) and a periodic
    stream are handed to the host library; the .lfm bytes stay identical."""
    torch = gpu
    runs4 = np.repeat(np.arange(190000 // 4, dtype=np.uint32) % 251, 4).astype(np.uint8)
    d = torch.from_numpy(runs4.copy()).cuda()
    got, flags = lfmlib.bzip2_device(d, [len(runs4), 1, 1, 1, 1], [len(runs4), 1, 1, 1, 1], 1, level=2)
    assert flags == [1] and got == [None]
    # through the encoder: the flagged streams are compressed on the host
    img = np.stack([runs4[:95000].reshape(1, 95000), np.tile(np.array([[3, 7]], np.uint8), (1, 47500))])
    img = img.reshape(1, 1, 2, 1, 95000)  # x = 95000, z = 2: two streams of one row each
    enc = lfmlib.Encoder(device=0)
    # device-resident (a host image this small goes to the host library whole)
    b, st = enc.encode(torch.from_numpy(img.copy()).cuda(), header_version=8, nnum=13,
                       block_size=[95000, 1, 1, 1, 1])
    enc.close()
    assert b == oracle.encode(img, header_version=8, nnum=13, data_type=0, block_size=[95000, 1, 1, 1, 1])


@pytest.mark.parametrize("W,H,T", [(200, 150, 13), (64, 70, 31), (45, 31, 5), (1, 1, 13), (300, 130, 15), (70, 90, 2),
                                   (33, 70, 1), (96, 600, 7), (136, 200, 30), (256, 330, 15)])
def test_unpredict_kernel_inverts_forward(lfmlib, oracle, gpu, W, H, T):
    """The GPU inverse returns the raw frames for every family and predictor
    (spatial), and for tiles video stacks (temporal odd frames); the oracle's
    forward symbols are the input."""
    torch = gpu
    stack = oracle.synthetic_lf(W, H, Z=4, T=T, seed=W * 3 + H)[0, 0]
    stack[1] = np.random.default_rng(W).integers(0, 65536, size=(H, W), dtype=np.uint16)  # int16 wrap
    for fam in FAMS:
        for k in range(1, 8):
            videos = (0, 1) if fam == "tiles" else (0,)
            for video in videos:
                sym = oracle.predict_volume(stack, T, fam, k, video)
                d_out = torch.empty((4, H, W), dtype=torch.int16, device="cuda")
                lfmlib.unpredict_device(dev16(torch, sym), d_out, W, H, 4, T, fam, k, video=video)
                torch.cuda.synchronize()
                assert np.array_equal(d_out.cpu().numpy().view(np.uint16), stack), (fam, k, video)


def test_unpredict_rejects_lossy_temporal(lfmlib, gpu):
    torch = gpu
    d = torch.zeros((2, 16, 16), dtype=torch.int16, device="cuda")
    with pytest.raises(lfmlib.LfmError):
        lfmlib.unpredict_device(d, d.clone(), 16, 16, 2, 13, "angle", 4, video=1)


@pytest.mark.parametrize("nfr", [1, 2, 3, 4, 5, 6, 7, 12])
def test_unpredict_band5_frame_counts(lfmlib, oracle, gpu, nfr):
    """The cross-workgroup inverse (band5: one single-wave workgroup per 64-row
    band, 5 bands of a 520 x 300 tiles frame) for every frame count, above all
    the counts that are not a multiple of 8 -- the round-5 hand-over timeout
    (GPUTEST_r05: 4 frames x 5 bands) came from such a launch.  Bands take
    their index from a ticket, not from blockIdx, so no count depends on the
    dispatch order or the XCD placement; the pixels are exact and no
    hand-over timed out (the call raises when one was not repaired)."""
    import time
    torch = gpu
    stack = oracle.synthetic_lf(520, 300, Z=nfr, T=13, seed=0x4C464D09 + nfr)[0, 0]
    for video in (0, 1):
        sym = oracle.predict_volume(stack, 13, "tiles", 5, video)
        d_sym = dev16(torch, sym)
        d_out = torch.empty_like(d_sym)
        t0 = time.time()
        for _ in range(3):  # repeated on the same control blocks
            d_out.zero_()
            lfmlib.unpredict_device(d_sym, d_out, 520, 300, nfr, 13, "tiles", 5, video=video)
            torch.cuda.synchronize()
            assert np.array_equal(host16(d_out), stack), (nfr, video)
        assert time.time() - t0 < 10.0


def test_unpredict_forced_timeout_is_bounded(lfmlib, oracle, gpu, capfd, monkeypatch):
    """A band5 hand-over forced to give up after one poll (LFM_UNPREDICT_SPIN=1)
    on a frame count that is not a multiple of 8: every band stops waiting
    once the status word carries the timeout, the device re-runs the frames
    through the one-wave kernel, and the call returns exact pixels within a second,
    reporting the timeout on stderr.  With LFM_UNPREDICT_FALLBACK=0 the same
    call fails instead of returning the pixels."""
    import time
    torch = gpu
    stack = oracle.synthetic_lf(520, 300, Z=4, T=13, seed=5)[0, 0]
    sym = oracle.predict_volume(stack, 13, "tiles", 5, 0)
    d_sym = dev16(torch, sym)
    d_out = torch.empty_like(d_sym)
    lfmlib.unpredict_device(d_sym, d_out, 520, 300, 4, 13, "tiles", 5)  # warm (module load)
    torch.cuda.synchronize()
    capfd.readouterr()
    monkeypatch.setenv("LFM_UNPREDICT_SPIN", "1")
    d_out.zero_()
    torch.cuda.synchronize()
    t0 = time.time()
    lfmlib.unpredict_device(d_sym, d_out, 520, 300, 4, 13, "tiles", 5)
    dt = time.time() - t0
    assert "hand-over timed out" in capfd.readouterr().err
    assert dt < 1.0, dt
    assert np.array_equal(host16(d_out), stack)
    monkeypatch.setenv("LFM_UNPREDICT_FALLBACK", "0")
    t0 = time.time()
    with pytest.raises(lfmlib.LfmError):
        lfmlib.unpredict_device(d_sym, d_out, 520, 300, 4, 13, "tiles", 5)
    assert time.time() - t0 < 1.0
    assert "not valid" in capfd.readouterr().err
    monkeypatch.delenv("LFM_UNPREDICT_SPIN")
    monkeypatch.delenv("LFM_UNPREDICT_FALLBACK")
    lfmlib.unpredict_device(d_sym, d_out, 520, 300, 4, 13, "tiles", 5)
    torch.cuda.synchronize()
    assert np.array_equal(host16(d_out), stack)
    assert "timed out" not in capfd.readouterr().err


def test_decode_roundtrip_through_gpu(lfmlib, oracle, gpu, tmp_path):
    """write (GPU predictor + GPU bzip2) -> read (bzip2 decode + GPU inverse)
    restores every pixel, video tiles stack included."""
    img = oracle.synthetic_lf(300, 200, Z=6, T=13, seed=77)
    for fam, hv in (("tiles", 0x80), ("angle", 0), ("space", 8 + 6)):
        lfmlib.set_family(fam)
        try:
            p = tmp_path / ("rt_%s.lfm" % fam)
            lfmlib.write_lfm(str(p), img, predictor_request=hv & 0x7F, nnum=13, video=hv >> 7)
            out, hv_out, nnum = lfmlib.read_lfm(str(p))
        finally:
            lfmlib.set_family("tiles")
        assert np.array_equal(out, img), fam


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(200, 136, 20), (256, 96, 16), (96, 96, 9)])
def test_decode_multilayer_roundtrip(lfmlib, oracle, gpu, tmp_path, shape):
    """Stacks of several block layers along z (ragged x / y blocks, an odd
    number of layers, a last layer of one frame) round-trip through the GPU
    writer and reader."""
    X, Y, Z = shape
    img = oracle.synthetic_lf(X, Y, Z=Z, T=13, seed=X + Z)
    for fam, hv in (("angle", 0), ("tiles", 8 + 2)):
        lfmlib.set_family(fam)
        try:
            p = tmp_path / ("layers_%s.lfm" % fam)
            lfmlib.write_lfm(str(p), img, predictor_request=hv & 0x7F, nnum=13, video=0)
            out, _, _ = lfmlib.read_lfm(str(p))
        finally:
            lfmlib.set_family("tiles")
        assert np.array_equal(out, img), (fam, shape)


@pytest.mark.gpu
def test_decode_roundtrip_5d_through_gpu(lfmlib, oracle, gpu, tmp_path):
    """5-D stacks (c, t > 1: one predictor volume per (c, t)) with small blocks
    round-trip through the GPU writer and reader (pipelined inverse predictor,
    W % 8 == 0), and ROI reads across c and t equal crops."""
    import ctypes
    img = oracle.synthetic_lf(256, 130, Z=4, C=2, Tn=3, T=13, seed=91)
    rng = np.random.default_rng(5)
    for fam, hv in (("tiles", 0x80 + 8 + 4), ("angle", 8 + 3)):
        lfmlib.set_family(fam)
        try:
            p = tmp_path / ("rt5_%s.lfm" % fam)
            lfmlib.write_lfm(str(p), img, predictor_request=hv & 0x7F, nnum=13, video=hv >> 7,
                             block_size=[64, 32, 2, 1, 1])
            out, _, _ = lfmlib.read_lfm(str(p))
            assert np.array_equal(out, img), fam
            for _ in range(4):
                lb, ub = [], []
                for d in (256, 130, 4, 2, 3):
                    a, b = sorted(int(v) for v in rng.integers(0, d, size=2))
                    lb.append(a)
                    ub.append(b)
                roi = np.empty(tuple(ub[d] - lb[d] + 1 for d in (4, 3, 2, 1, 0)), np.uint16)
                rc = lfmlib.lib().readKLBroiInPlace(os.fsencode(str(p)), roi.ctypes.data, (ctypes.c_uint32 * 5)(*lb),
                                                     (ctypes.c_uint32 * 5)(*ub), 4)
                assert rc == 0
                want = img[lb[4]:ub[4] + 1, lb[3]:ub[3] + 1, lb[2]:ub[2] + 1, lb[1]:ub[1] + 1, lb[0]:ub[0] + 1]
                assert np.array_equal(roi, want), (fam, lb, ub)
        finally:
            lfmlib.set_family("tiles")


@pytest.mark.gpu
def test_gpu_bunzip2_matches_libbz2(lfmlib, oracle, gpu):
    """GPU bzip2 decoder on streams of the reference's bzip2-1.0.6:
    streams of every level,
    long runs (RLE1 count bytes, RUNA/RUNB), random and periodic data, tiny
    blocks; a two-block stream and a damaged stream are flagged for the host."""
    rng = np.random.default_rng(7)
    cases = []
    for level in (1, 2, 5, 9):
        cases.append((rng.integers(0, 256, 90000, dtype=np.uint8).tobytes(), level))
    cases += [
        (bytes(150000), 2),                                        # one long run
        (b"\x07" * 5 + b"ab" * 300 + b"\x00" * 1000, 1),          # runs of 4+, periodic
        (rng.integers(0, 4, 140000, dtype=np.uint8).tobytes(), 2),  # small alphabet
        ((np.arange(147456) % 251).astype(np.uint8).tobytes(), 2),
        (b"x", 1),
        (b"hello, light field", 9),
        (rng.integers(0, 2, 150000, dtype=np.uint8).repeat(3)[:147456].tobytes(), 2),
    ]
    streams = [ref_bz2(oracle, d, lv) for d, lv in cases]
    out, flags = lfmlib.bunzip2_device(streams, 160000)
    for (d, lv), o, f in zip(cases, out, flags):
        assert f == 0, (lv, len(d), f)
        assert o == d, (lv, len(d))
    # two bzip2 blocks (more than 100k after RLE1 at level 1) -> host; a flipped bit -> not accepted
    big = rng.integers(0, 256, 150000, dtype=np.uint8).tobytes()
    bad = bytearray(ref_bz2(oracle, b"some data to damage" * 100, 1))
    bad[len(bad) // 2] ^= 0x10
    out, flags = lfmlib.bunzip2_device([ref_bz2(oracle, big, 1), bytes(bad)], 160000)
    assert flags[0] == 1 and out[0] is None
    assert flags[1] != 0 and out[1] is None


def test_roi_read_small_blocks_gpu(lfmlib, oracle, gpu, tmp_path):
    """ROI reads of predicted files with many blocks (only the blocks up / left
    of the ROI decoded, on the GPU path) equal the crop of the image: every
    family at predictor 4, and a tiles video stack (odd first frames)."""
    import ctypes
    rng = np.random.default_rng(11)
    img = oracle.synthetic_lf(150, 110, Z=6, T=13, seed=0x4C464D07)[0, 0]
    cases = [("tiles", 0), ("angle", 0), ("space", 0), ("tiles", 1)]
    for fam, video in cases:
        p = tmp_path / ("roi_%s_%d.lfm" % (fam, video))
        lfmlib.write_lfm(str(p), img, predictor_request=8 + 4, nnum=13, video=video, block_size=[32, 24, 2, 1, 1],
                         family=fam)
        try:
            for _ in range(6):
                lb, ub = [], []
                for d in (150, 110, 6, 1, 1):
                    a, b = sorted(int(v) for v in rng.integers(0, d, size=2))
                    lb.append(a)
                    ub.append(b)
                out = np.empty((ub[2] - lb[2] + 1, ub[1] - lb[1] + 1, ub[0] - lb[0] + 1), np.uint16)
                rc = lfmlib.lib().readKLBroiInPlace(os.fsencode(str(p)), out.ctypes.data, (ctypes.c_uint32 * 5)(*lb),
                                                     (ctypes.c_uint32 * 5)(*ub), 4)
                assert rc == 0
                assert np.array_equal(out, img[lb[2]:ub[2] + 1, lb[1]:ub[1] + 1, lb[0]:ub[0] + 1]), (fam, video, lb, ub)
        finally:
            lfmlib.set_family("tiles")


def test_pipelined_submit_wait(lfmlib, oracle, gpu):
    """lfm_encoder_submit / lfm_encoder_wait: two encodes in flight (the
    second builds while the first's payload copies run) give the same bytes as
    synchronous encodes of the same stacks -- stacks and slabs, device and host
    input; a ticket two submits old is refused; a synchronous encode after
    submits still works."""
    torch = gpu
    stacks = [oracle.synthetic_lf(480, 400, Z=24, T=15, seed=100 + i)[0, 0] for i in range(4)]
    lfmlib.set_family("angle")
    try:
        sync = lfmlib.Encoder(device=0)
        exp = [sync.encode(s, header_version=0, nnum=15)[0] for s in stacks]
        exp_slab = sync.encode_slab(stacks[0][8:], 8, header_version=8 + 4, nnum=15)[0]
        sync.close()
        enc = lfmlib.Encoder(device=0)
        tickets = []
        got = {}
        for i, s in enumerate(stacks):
            img = dev16(torch, s) if i % 2 == 0 else s
            tickets.append(enc.submit(img, header_version=0, nnum=15))
            del img
            if i >= 1:
                got[i - 1] = enc.wait(tickets[i - 1])[0]
        got[3] = enc.wait(tickets[3])[0]
        assert [got[i] for i in range(4)] == exp
        assert enc.wait(tickets[3])[0] == exp[3]  # waiting twice is fine
        with pytest.raises(lfmlib.LfmError):
            enc.wait(tickets[1])  # two submits ago: its buffers are reused
        t = enc.submit(dev16(torch, stacks[0][8:]), z0=8, header_version=8 + 4, nnum=15)
        b, st = enc.wait(t)
        assert b == exp_slab and st["out_bytes"] == len(b)
        b2, _ = enc.encode(stacks[1], header_version=0, nnum=15)
        assert b2 == exp[1]
        enc.close()
    finally:
        lfmlib.set_family("tiles")


_UPLOAD_CHILD = r"""
import json, sys
import numpy as np
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
import torch, lfm, lfm_oracle as O
torch.cuda.set_device(0)
out = {}
enc = lfm.Encoder(device=0)
# 1. tiles video stack: 1-MiB chunks (4 frames of 512 x 256), a 2-MiB ring
#    (3 slots, the minimum: every slot reused, temporal predecessors across
#    chunk edges)
img = O.synthetic_lf(512, 256, Z=21, T=13, seed=41)
lfm.set_family("tiles")
out["video"] = enc.encode(img, header_version=0x80, nnum=13)[0] == O.encode(img, header_version=0x80, nnum=13,
                                                                               family="tiles")
# 2. 5-D stack (c = 2, t = 3): chunks never cross a (c, t) volume
img5 = O.synthetic_lf(520, 200, Z=5, C=2, Tn=3, T=15, seed=42)
out["5d"] = enc.encode(img5, header_version=8 + 5, nnum=15, block_size=[64, 64, 2, 1, 1])[0] == O.encode(
    img5, header_version=8 + 5, nnum=15, family="tiles", block_size=[64, 64, 2, 1, 1])
# 3. a z-slab of a video stack starting at an odd frame, host input: its
#    previous raw frame comes from the host; the second slab's 24 frames are
#    6 chunks, so the ring's slots are reused under the odd-start pairing
full = O.synthetic_lf(512, 256, Z=33, T=13, seed=43)[0, 0]
k, _ = lfm.select_device(torch.from_numpy(full[0].view(np.int16)).cuda(), 512, 256, 13, "tiles")
bs = [64, 64, 3, 1, 1]
a, _ = enc.encode_slab(full[:9], 0, header_version=0x80 | (8 + k), nnum=13, block_size=bs)
b, _ = enc.encode_slab(full[9:], 9, prev=full[8], header_version=0x80 | (8 + k), nnum=13, block_size=bs)
out["slab"] = lfm.merge_slabs([a, b]) == O.encode(full, header_version=0x80, nnum=13, family="tiles",
                                                  block_size=bs)
# 4. pipelined host submits: after submit returns the stack may be refilled
stacks = [O.synthetic_lf(512, 256, Z=16, T=15, seed=50 + i)[0, 0] for i in range(3)]
lfm.set_family("angle")
exp = [O.encode(s.copy(), header_version=0, nnum=15, family="angle") for s in stacks]
buf = np.empty_like(stacks[0])
got, prev = [], None
for s in stacks:
    buf[...] = s
    t = enc.submit(buf, header_version=0, nnum=15)
    buf[...] = 0x1234  # the upload is complete when submit returns
    if prev is not None:
        got.append(enc.wait(prev)[0])
    prev = t
got.append(enc.wait(prev)[0])
out["pipelined"] = got == exp
enc.close()
print(json.dumps(out))
"""


def test_host_upload_pipe_chunks_and_ring(gpu, tmp_path):
    """Host stacks upload in chunks through a ring of device slots, each chunk
    predicted as it lands and every GPU-bzip2 batch waiting only for its
    chunks (UploadPipe).  With 1-MiB chunks and a 3-slot ring every slot is
    reused: video stacks (temporal predecessors across chunk edges), 5-D
    stacks, an odd-start video slab with its previous frame from the host, and
    pipelined host submits (the stack refilled as soon as submit returns)
    give the oracle's bytes."""
    import subprocess
    import sys
    from conftest import PKG, REPO
    env = dict(os.environ, LFM_H2D_CHUNK_MB="1", LFM_H2D_RING_MB="2")
    r = subprocess.run([sys.executable, "-c", _UPLOAD_CHILD, PKG, os.path.join(REPO, "oracle")], env=env,
                       capture_output=True, text=True, timeout=200)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert got == {"video": True, "5d": True, "slab": True, "pipelined": True}, got


def test_submit_releases_unpredicted_device_input(lfmlib, oracle, gpu):
    """A submit whose stack skips the predictor stage (forced predictor 0,
    request 8) returns with the caller's device image no longer referenced:
    overwriting the tensor before wait() must not change the .lfm."""
    torch = gpu
    stack = oracle.synthetic_lf(480, 400, Z=16, T=15, seed=77)[0, 0]
    exp = oracle.encode(stack, header_version=8, nnum=15, family="tiles")
    enc = lfmlib.Encoder(device=0)
    try:
        d = dev16(torch, stack)
        t = enc.submit(d, header_version=8, nnum=15)
        d.fill_(0x1234)  # a camera ring buffer refilling the slot
        torch.cuda.synchronize()
        b, st = enc.wait(t)
        assert b == exp and st["chosen"] == 0
    finally:
        enc.close()


def test_submit_select_frame_and_wait_codes(lfmlib, oracle, gpu):
    """Auto-selection inside submit on a slab: select_frame = the whole
    stack's frame 0 makes every slab select what the whole stack selects
    (bytes equal the forced-slab encode); an auto slab without it is refused;
    waiting on a ticket never issued returns code 8 and no buffer."""
    import ctypes
    torch = gpu
    stack = oracle.synthetic_lf(480, 400, Z=24, T=15, seed=5150)[0, 0]
    lfmlib.set_family("angle")
    try:
        k, _ = oracle.select(stack[0], 15, "angle")
        exp = oracle.encode(stack[8:], header_version=8 + k, nnum=15, family="angle", z0=8)
        enc = lfmlib.Encoder(device=0)
        d = dev16(torch, stack)
        t = enc.submit(d[8:], z0=8, header_version=0, nnum=15, select_frame=d[0])
        b, st = enc.wait(t)
        assert b == exp and st["chosen"] == k and st["select_ms"] > 0
        # the same from host memory
        t = enc.submit(stack[8:], z0=8, header_version=0, nnum=15, select_frame=stack[0])
        assert enc.wait(t)[0] == exp
        with pytest.raises(lfmlib.LfmError):
            enc.submit(d[8:], z0=8, header_version=0, nnum=15)
        with pytest.raises(lfmlib.LfmError):  # (the synchronous slab entry refuses it too)
            enc.encode_slab(d[8:], 8, prev=d[7], header_version=0, nnum=15)
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_uint64(123)
        rc = lfmlib.lib().lfm_encoder_wait(enc._h, 987654321, ctypes.byref(out), ctypes.byref(n), None)
        assert rc == 8 and not out and n.value == 0
        enc.close()
    finally:
        lfmlib.set_family("tiles")


@pytest.mark.parametrize("env", ["LFM_DECODE_H2D=1", "LFM_DECODE_H2D=2"])
def test_decode_path_switches(lfmlib, oracle, gpu, tmp_path, env):
    """The decode's fallback payload uploads (one runtime copy, or
    hipMemcpyAsync from the pinned chunks, instead of the SDMA engine) restore
    the same pixels.  The switches are read once per process: each variant
    decodes in its own child process (one GPU process at a time)."""
    import subprocess
    import sys
    from conftest import PKG
    img = oracle.synthetic_lf(256, 192, Z=16, T=13, seed=5)
    lfmlib.set_family("angle")
    try:
        p = tmp_path / "sw.lfm"
        lfmlib.write_lfm(str(p), img, predictor_request=0, nnum=13, video=0)
    finally:
        lfmlib.set_family("tiles")
    out = tmp_path / "out.npy"
    code = ("import sys; sys.path.insert(0, %r); import numpy as np, lfm; lfm.set_family('angle'); "
            "o, _, _ = lfm.read_lfm(%r); np.save(%r, o)" % (PKG, str(p), str(out)))
    child_env = dict(os.environ)
    child_env.update(kv.split("=", 1) for kv in env.split())
    r = subprocess.run([sys.executable, "-c", code], env=child_env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    assert np.array_equal(np.load(out).reshape(img.shape), img), env


@pytest.mark.parametrize("env", ["LFM_DECODE_CHUNK_BLOCKS=1", "LFM_DECODE_CHUNK_BLOCKS=1 LFM_DECODE_SLOTS=3",
                                 "LFM_DECODE_CHUNK_BLOCKS=0", "LFM_DECODE_CHUNK_BLOCKS=1 LFM_DECODE_H2D=2"])
def test_decode_chunk_pipeline(lfmlib, oracle, gpu, tmp_path, env):
    """The pipelined GPU decode (chunks of whole block slabs on 2-3 HIP
    streams, downloads on their own thread) restores the pixels whatever the
    chunking: one slab per chunk on a video tiles stack of two t-volumes with
    3-frame blocks puts chunk starts on odd (temporal) frames, whose previous
    frame comes from the chunk before (event hand-over), and on volume starts;
    one chunk; the hipMemcpyAsync upload.  Each variant runs in its own child
    process (the switches are read once per process)."""
    import subprocess
    import sys
    from conftest import PKG
    img = oracle.synthetic_lf(200, 136, Z=10, C=1, Tn=2, T=13, seed=77)
    lfmlib.set_family("tiles")
    p = tmp_path / "ck.lfm"
    lfmlib.write_lfm(str(p), img, predictor_request=8 + 4, nnum=13, video=1, block_size=[64, 64, 3, 1, 1])
    out = tmp_path / "out.npy"
    code = ("import sys; sys.path.insert(0, %r); import numpy as np, lfm; lfm.set_family('tiles'); "
            "o, _, _ = lfm.read_lfm(%r); np.save(%r, o)" % (PKG, str(p), str(out)))
    child_env = dict(os.environ)
    child_env.update(kv.split("=", 1) for kv in env.split())
    r = subprocess.run([sys.executable, "-c", code], env=child_env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    assert np.array_equal(np.load(out).reshape(img.shape), img), env


@pytest.mark.parametrize("fallback", [True, False])
def test_unpredict_band_timeout_is_reported(lfmlib, oracle, gpu, tmp_path, fallback):
    """A band of the cross-CU inverse predictor (band5) that gives up waiting
    for the band above (here forced: one poll, LFM_UNPREDICT_SPIN=1) sets the
    launch's error word: the device re-runs the frames (one-wave kernel) and the
    pixels are exact, or with LFM_UNPREDICT_FALLBACK=0 the read fails -- never
    wrong pixels returned as success."""
    import subprocess
    import sys
    from conftest import PKG
    img = oracle.synthetic_lf(256, 192, Z=16, T=13, seed=6)
    lfmlib.set_family("tiles")
    p = tmp_path / "to.lfm"
    lfmlib.write_lfm(str(p), img, predictor_request=8 + 4, nnum=13, video=1)
    out = tmp_path / "out.npy"
    code = ("import sys; sys.path.insert(0, %r); import numpy as np, lfm; lfm.set_family('tiles'); "
            "o, _, _ = lfm.read_lfm(%r); np.save(%r, o)" % (PKG, str(p), str(out)))
    child_env = dict(os.environ, LFM_UNPREDICT_SPIN="1", LFM_UNPREDICT_FALLBACK="1" if fallback else "0")
    r = subprocess.run([sys.executable, "-c", code], env=child_env, capture_output=True, text=True, timeout=110)
    assert "hand-over timed out" in r.stderr, r.stderr[-2000:]
    if fallback:
        assert r.returncode == 0, r.stderr[-2000:]
        assert np.array_equal(np.load(out).reshape(img.shape), img)
    else:
        assert r.returncode != 0 and not out.exists()


def test_decode_threads_release_device_memory(lfmlib, oracle, gpu, tmp_path):
    """Decodes from short-lived host threads free their per-thread device
    buffers and pinned staging when the thread exits: the
    device's free memory does not shrink with the number of threads."""
    import threading
    torch = gpu
    img = oracle.synthetic_lf(1024, 1024, Z=16, T=13, seed=9)
    p = tmp_path / "thr.lfm"
    lfmlib.write_lfm(str(p), img, predictor_request=8 + 4, nnum=13)
    buf = p.read_bytes()
    errors = []

    def one():
        try:
            if not np.array_equal(lfmlib.decode(buf).reshape(img.shape), img):
                errors.append("pixels")
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e))

    def run_thread():
        th = threading.Thread(target=one)
        th.start()
        th.join()

    run_thread()
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(6):
        run_thread()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert not errors, errors
    assert free0 - free1 < (128 << 20), (free0, free1)


def test_encoder_rejects_bad_device_operands(lfmlib, gpu):
    """Encoder._operand: strided views and unsupported dtypes
    are refused instead of encoding the wrong pixels."""
    torch = gpu
    enc = lfmlib.Encoder(device=torch.cuda.current_device())
    try:
        d = torch.zeros((8, 64, 128), dtype=torch.int16, device="cuda")
        with pytest.raises(lfmlib.LfmError):
            enc.encode(d[:, :, ::2], nnum=13)
        with pytest.raises(lfmlib.LfmError):
            enc.encode(torch.zeros((8, 64, 64), dtype=torch.float16, device="cuda"), nnum=13)
    finally:
        enc.close()


@pytest.mark.parametrize("fam", ["angle", "space"])
def test_video_with_lossy_family_reads_loudly(lfmlib, oracle, gpu, tmp_path, fam):
    """Video stacks with the angle / space families: the writer reproduces the
    reference's bytes (with a warning: its temporal residual drops a bit) and
    the reader refuses the file with an error instead of returning wrong
    pixels."""
    img = oracle.synthetic_lf(96, 96, Z=4, T=13, seed=3)
    lfmlib.set_family(fam)
    try:
        p = tmp_path / "v.lfm"
        lfmlib.write_lfm(str(p), img, predictor_request=8 + 4, nnum=13, video=1)
        with pytest.raises(lfmlib.LfmError):
            lfmlib.read_lfm(str(p))
    finally:
        lfmlib.set_family("tiles")
