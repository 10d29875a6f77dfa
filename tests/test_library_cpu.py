"""CPU-only tests of liblfm.so: it loads, exports every declared symbol, and
its host paths (container, block scheduler, bzip2/zlib, decoder) match the oracle."""
import hashlib
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, REPO

INCLUDE = os.path.join(REPO, "include", "lfm")


def declared_c_functions():
    names = set()
    for h in ("klb_Cwrapper.h", "lfm_api.h", "lfm_hip.h"):
        src = open(os.path.join(INCLUDE, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:DECLSPECIFIER|LFM_API)?\s*[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", src, re.M):
            name = m.group(1)
            if name in ("if", "defined", "__attribute__", "visibility"):
                continue
            names.add(name)
    return sorted(names)


def test_library_exports_every_declared_symbol(lfmlib):
    L = lfmlib.lib()
    decl = declared_c_functions()
    assert "writeKLBstack" in decl and "lfm_hip_predict" in decl and "lfm_encoder_encode" in decl
    missing = [n for n in decl if not hasattr(L, n)]
    assert missing == []
    assert lfmlib.missing_exports() == []
    assert b"gfx950" in L.lfm_version()


def test_cpp_class_symbols_exported(lfmlib):
    """klb_imageIO / klb_image_header (the MEX link surface) are exported."""
    import subprocess
    out = subprocess.run(["nm", "-DC", lfmlib.LIB_PATH], capture_output=True, text=True).stdout
    for sym in ("klb_imageIO::writeImage(char const*, int)", "klb_imageIO::readImageFull(char*, int)",
                "klb_image_header::setDefaultBlockSize()", "klb_image_header::writeHeader(_IO_FILE*)",
                "klb_imageIO::readImage(char*, klb_ROI const*, int)"):
        assert sym in out, sym


def _img_tif():
    return np.load(os.path.join(GOLDEN, "img_tif.npz"))["img"]


def _manifest():
    return {e["name"]: e for e in json.load(open(os.path.join(GOLDEN, "lfm_manifest.json")))}


def test_config1_plumbing_bit_identical(lfmlib, tmp_path):
    """Config 1: img.tif page 0 (all zeros), request 8 (predictor off), default
    blocks, BZIP2 on the CPU: identical bytes to the oracle's file."""
    man = _manifest()
    img = _img_tif()
    for name, arr in (("cfg1_imgtif_page0_req8", img[0]), ("cfg1_imgtif_stack_req8", img)):
        p = tmp_path / (name + ".lfm")
        lfmlib.write_lfm(p, arr, predictor_request=8, nnum=13)
        b = p.read_bytes()
        assert hashlib.sha256(b).hexdigest() == man[name]["sha256"], name
        back, hv, nn = lfmlib.read_lfm(p)
        assert np.array_equal(back.reshape(arr.shape), arr) and hv == 0 and nn == 13


def test_writeKLBstack_defaults_and_readKLB(lfmlib, tmp_path, oracle):
    """writeKLBstack on 8-bit data: no predictor stage (16-bit only), default blocks."""
    rng = np.random.default_rng(1)
    arr = rng.integers(0, 8, size=(3, 50, 70), dtype=np.uint8)
    p = tmp_path / "u8.klb"
    lfmlib.write_klb(p, arr, metadata="hello")
    h = lfmlib.read_header(p)
    assert h["xyzct"] == [70, 50, 3, 1, 1] and h["data_type"] == 0 and h["block_size"] == [70, 50, 3, 1, 1]
    assert h["metadata"].startswith(b"hello\0")
    assert p.read_bytes() == oracle.encode(arr, header_version=0, data_type=0, metadata=b"hello")
    back, hv, _ = lfmlib.read_lfm(p)
    assert np.array_equal(back.reshape(arr.shape), arr)


@pytest.mark.parametrize("dtype,dt", [(np.float32, 8), (np.int32, 6), (np.uint64, 3)])
def test_wide_types_roundtrip(lfmlib, tmp_path, oracle, dtype, dt):
    rng = np.random.default_rng(2)
    arr = (rng.random((2, 3, 4, 33, 47)) * 100).astype(dtype)
    p = tmp_path / "w.lfm"
    lfmlib.write_lfm(p, arr, predictor_request=0, block_size=[16, 16, 3, 2, 1])
    assert p.read_bytes() == oracle.encode(arr, header_version=0, data_type=dt, block_size=[16, 16, 3, 2, 1])
    back, _, _ = lfmlib.read_lfm(p)
    assert np.array_equal(back.reshape(arr.shape), arr)


def test_ragged_blocks_5d_raw(lfmlib, tmp_path, oracle):
    """5-D image, border blocks on every axis, request 8: bytes match the oracle."""
    img = oracle.synthetic_lf(37, 29, Z=5, C=2, Tn=3, T=7)
    p = tmp_path / "r.lfm"
    lfmlib.write_lfm(p, img, predictor_request=8, nnum=7, block_size=[16, 8, 2, 1, 2])
    assert p.read_bytes() == oracle.encode(img, header_version=8, nnum=7, block_size=[16, 8, 2, 1, 2])
    back, _, _ = lfmlib.read_lfm(p)
    assert np.array_equal(back, img)


def test_compression_none_and_zlib(lfmlib, tmp_path, oracle):
    img = oracle.synthetic_lf(40, 30, Z=2, T=13)
    for ct in (0, 2):
        p = tmp_path / ("c%d.lfm" % ct)
        lfmlib.write_lfm(p, img, predictor_request=8, compression=ct)
        if ct == 0:
            assert p.read_bytes() == oracle.encode(img, header_version=8, compression=0)
        back, _, _ = lfmlib.read_lfm(p)
        assert np.array_equal(back, img)


def test_decode_committed_predictor_files(lfmlib):
    """The product decoder inverts the committed oracle .lfm files (all
    families, all forced predictors) back to their generator input."""
    import lfm_oracle as O
    man = _manifest()
    small = O.synthetic_lf(70, 45, Z=3, T=13, seed=0x4C464D06)
    for fam in ("tiles", "angle", "space"):
        lfmlib.set_family(fam)
        try:
            for k in range(8):
                e = man["small_%s_req%d" % (fam, 8 + k)]
                b = open(os.path.join(GOLDEN, e["file"]), "rb").read()
                out = lfmlib.decode(b)
                assert np.array_equal(out, small), (fam, k)
        finally:
            lfmlib.set_family("tiles")


def test_decode_video_tiles_file(lfmlib):
    man = _manifest()
    b = open(os.path.join(GOLDEN, man["imgtif_stack_auto_video"]["file"]), "rb").read()
    out = lfmlib.decode(b)
    assert np.array_equal(out.reshape(_img_tif().shape), _img_tif())


def test_roi_read(lfmlib, tmp_path):
    import ctypes
    man = _manifest()
    p = os.path.join(GOLDEN, man["imgtif_stack_auto_video"]["file"])
    img = _img_tif()
    lb, ub = [10, 20, 3, 0, 0], [60, 100, 9, 0, 0]
    out = np.empty((7, 81, 51), np.uint16)
    rc = lfmlib.lib().readKLBroiInPlace(os.fsencode(p), out.ctypes.data, (ctypes.c_uint32 * 5)(*lb),
                                         (ctypes.c_uint32 * 5)(*ub), 2)
    assert rc == 0
    assert np.array_equal(out, img[3:10, 20:101, 10:61])


def _read_roi(lfmlib, path, lb, ub, dtype=np.uint16):
    import ctypes
    shape = tuple(ub[d] - lb[d] + 1 for d in (4, 3, 2, 1, 0))
    out = np.empty(shape, dtype)
    rc = lfmlib.lib().readKLBroiInPlace(os.fsencode(str(path)), out.ctypes.data, (ctypes.c_uint32 * 5)(*lb),
                                         (ctypes.c_uint32 * 5)(*ub), 2)
    assert rc == 0, (lb, ub)
    return out


def _rois(dims, rng, n):
    """ROIs over xyzct dims: the whole image, the last pixel, and n random boxes."""
    yield [0] * 5, [d - 1 for d in dims]
    yield [d - 1 for d in dims], [d - 1 for d in dims]
    for _ in range(n):
        lb, ub = [], []
        for d in dims:
            a, b = sorted(int(v) for v in rng.integers(0, d, size=2))
            lb.append(a)
            ub.append(b)
        yield lb, ub


def test_roi_reads_match_crop_of_full_decode(lfmlib, tmp_path):
    """ROI reads decode only the blocks the ROI depends on (everything up / left
    in its frames with predictors, the frame before an odd frame of a video
    stack) and must equal the crop of the full image: predicted files of every
    family, the video stack, and a 5-D raw file with border blocks on every axis."""
    import lfm_oracle as O
    man = _manifest()
    rng = np.random.default_rng(7)
    small = O.synthetic_lf(70, 45, Z=3, T=13, seed=0x4C464D06)
    for fam in ("tiles", "angle", "space"):
        lfmlib.set_family(fam)
        try:
            for k in (1, 4, 7):
                p = os.path.join(GOLDEN, man["small_%s_req%d" % (fam, 8 + k)]["file"])
                for lb, ub in _rois([70, 45, 3, 1, 1], rng, 4):
                    got = _read_roi(lfmlib, p, lb, ub)
                    want = small.reshape(1, 1, 3, 45, 70)[lb[4]:ub[4] + 1, lb[3]:ub[3] + 1, lb[2]:ub[2] + 1,
                                                          lb[1]:ub[1] + 1, lb[0]:ub[0] + 1]
                    assert np.array_equal(got, want), (fam, k, lb, ub)
        finally:
            lfmlib.set_family("tiles")
    img = _img_tif()
    p = os.path.join(GOLDEN, man["imgtif_stack_auto_video"]["file"])
    Z, Y, X = img.shape
    for lb, ub in _rois([X, Y, Z, 1, 1], rng, 6):
        got = _read_roi(lfmlib, p, lb, ub)
        assert np.array_equal(got[0, 0], img[lb[2]:ub[2] + 1, lb[1]:ub[1] + 1, lb[0]:ub[0] + 1]), (lb, ub)
    img5 = O.synthetic_lf(37, 29, Z=5, C=2, Tn=3, T=7)
    p5 = tmp_path / "r5.lfm"
    lfmlib.write_lfm(p5, img5, predictor_request=8, nnum=7, block_size=[16, 8, 2, 1, 2])
    for lb, ub in _rois([37, 29, 5, 2, 3], rng, 8):
        got = _read_roi(lfmlib, p5, lb, ub)
        want = img5[lb[4]:ub[4] + 1, lb[3]:ub[3] + 1, lb[2]:ub[2] + 1, lb[1]:ub[1] + 1, lb[0]:ub[0] + 1]
        assert np.array_equal(got, want), (lb, ub)


def test_decode_memory_roi_into_caller_buffer(lfmlib):
    """lfm_decode_memory_roi (lfm.decode_roi) on an in-memory .lfm: whole
    t-volumes and a sub-box equal the crop of the image, decoded into a fresh
    array or into a caller buffer reused across calls; a buffer of the wrong
    size or type is refused before anything is written."""
    man = _manifest()
    b = open(os.path.join(GOLDEN, man["imgtif_stack_auto_video"]["file"]), "rb").read()
    img = _img_tif()
    Z, Y, X = img.shape
    whole = lfmlib.decode_roi(b, [0, 0, 0, 0, 0], [X - 1, Y - 1, Z - 1, 0, 0])
    assert np.array_equal(whole.reshape(img.shape), img)
    buf = np.zeros((5, 40, 30), np.uint16)
    for z0 in (0, 3, Z - 5):
        got = lfmlib.decode_roi(b, [7, 11, z0, 0, 0], [36, 50, z0 + 4, 0, 0], out=buf)
        assert got.base is buf or got is buf
        assert np.array_equal(buf, img[z0:z0 + 5, 11:51, 7:37]), z0
    with pytest.raises(ValueError):
        lfmlib.decode_roi(b, [0, 0, 0, 0, 0], [9, 9, 0, 0, 0], out=np.zeros((10, 11), np.uint16))
    with pytest.raises(ValueError):
        lfmlib.decode_roi(b, [0, 0, 0, 0, 0], [9, 9, 0, 0, 0], out=np.zeros((10, 10), np.int32))


def test_decode_roi_uses_the_file_dtype(lfmlib, tmp_path):
    """decode_roi sizes its output from the header's data type (a uint32 or
    float32 .lfm read with default arguments), refuses an explicit dtype the
    file does not hold, and lfm_decode_memory_roi refuses an output buffer
    smaller than region x bytes per pixel instead of writing past it."""
    import ctypes
    rng = np.random.default_rng(3)
    for dt in (np.uint32, np.float32):
        img = (rng.integers(0, 1 << 20, (3, 20, 24)) if dt == np.uint32 else rng.random((3, 20, 24))).astype(dt)
        p = tmp_path / ("roi_%s.klb" % np.dtype(dt).name)
        lfmlib.write_klb(p, img)
        b = open(p, "rb").read()
        got = lfmlib.decode_roi(b, [2, 3, 1, 0, 0], [20, 17, 2, 0, 0])
        assert got.dtype == dt
        assert np.array_equal(got.reshape(2, 15, 19), img[1:3, 3:18, 2:21])
        with pytest.raises(ValueError):
            lfmlib.decode_roi(b, [0, 0, 0, 0, 0], [3, 3, 0, 0, 0], dtype=np.uint16)
        small = np.zeros(16, np.uint16)  # 4 x 4 pixels of 4 bytes need 64 bytes, not 32
        arr5 = (ctypes.c_uint32 * 5)
        rc = lfmlib.lib().lfm_decode_memory_roi(b, len(b), arr5(0, 0, 0, 0, 0), arr5(3, 3, 0, 0, 0),
                                                small.ctypes.data, small.nbytes, 1)
        assert rc == 3 and not small.any()
        rc = lfmlib.lib().lfm_decode_memory_roi(b, len(b), arr5(0, 0, 0, 0, 0), arr5(24, 3, 0, 0, 0),
                                                small.ctypes.data, 1 << 20, 1)
        assert rc == 3  # x = 24 is outside the 24-pixel rows


def test_invalid_predictor_request_rejected(lfmlib, tmp_path):
    img = np.zeros((1, 16, 16), np.uint16)
    with pytest.raises(lfmlib.LfmError, match="code 6"):
        lfmlib.write_lfm(tmp_path / "bad.lfm", img, predictor_request=16)


def test_gpu_required_for_predictor_stage(lfmlib, tmp_path):
    if lfmlib.device_count() > 0:
        pytest.skip("a GPU is visible")
    img = np.ones((1, 16, 16), np.uint16)
    with pytest.raises(lfmlib.LfmError, match="code 7"):
        lfmlib.write_lfm(tmp_path / "x.lfm", img, predictor_request=0)
    with pytest.raises(lfmlib.LfmError, match="code 7"):
        lfmlib.write_lfm(tmp_path / "y.lfm", img, predictor_request=9)


def test_unopenable_output(lfmlib):
    with pytest.raises(lfmlib.LfmError, match="code 5"):
        lfmlib.write_lfm("/nonexistent_dir/x.lfm", np.zeros((4, 4), np.uint16), predictor_request=8)


def test_family_switch(lfmlib):
    assert lfmlib.get_family() == 0
    lfmlib.set_family("space")
    assert lfmlib.get_family() == 2
    lfmlib.set_family("tiles")
    with pytest.raises(lfmlib.LfmError):
        lfmlib.set_family(5)


def test_band5_release_wait_covers_the_round_stores():
    """The inverse predictor's band hand-over publishes progress after a
    hand-counted `s_waitcnt vmcnt(2)` (3 on temporal frames): compile
    unpredict_band5 (one predictor per family) to gfx950 assembly and check,
    on the loop's back edge, that at least that many vector memory
    instructions follow the second-to-last round's pixel store -- so the wait
    proves every store but the last round's complete, whatever order the
    compiler chose (scripts/check_band5_isa.py)."""
    import subprocess
    import sys
    sys.path.insert(0, os.path.join(REPO, "scripts"))
    import check_band5_isa as C
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, "b5.s")
        try:
            C.compile_asm(asm)
        except (OSError, subprocess.CalledProcessError) as e:
            pytest.skip("hipcc unavailable: %s" % e)
        res = C.check(asm)
    waits = {(k, n) for k, n, _ in res}
    assert {n for _, n in waits} == {2, 3}, res           # both the spatial and the temporal wait
    assert len({k for k, _ in waits}) == 3, res           # in each family's kernel
    assert all(ops >= n for _, n, ops in res), res


def test_header_u64_offsets_past_4gib(oracle, tmp_path):
    """Block end-offsets past 2^32 (a 100-volume config-5 .lfm is 51.6 GB):
    liblfm's klb_image_header writes them as u64 (klb_imageHeader.h:46,
    klb_imageIO.cpp:1215-1217) and reads them back through readHeader,
    parseHeader and readKLBheader (tests/c/header_u64.cpp); the header bytes
    equal the oracle's and, when built, the reference class's own."""
    import ctypes
    import subprocess
    exe = os.path.join(REPO, "tests", "c", "header_u64")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.join(REPO, "tests", "c")], check=True, capture_output=True)
    path = str(tmp_path / "h64.lfm")
    r = subprocess.run([exe, path], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    b = open(path, "rb").read()
    xyzct, bs = [4096, 4096, 32, 1, 100], [96, 96, 8, 1, 1]
    nb = 43 * 43 * 4 * 100
    i = np.arange(nb, dtype=np.uint64)
    offs = np.cumsum(70000 + (i * 7919) % 5003).astype(np.uint64)
    assert int(offs[-1]) > 1 << 32 and len(b) == 320 + 8 * nb
    assert np.array_equal(np.frombuffer(b, "<u8", nb, 320), offs)
    md = b"u64 offsets".ljust(256, b"\0")
    assert b == oracle.header_bytes(0x84, 13, xyzct, [1, 1, 2.5, 1, 1], 1, 1, md, bs, offs)
    ref = os.path.join(REPO, "oracle", "_ref", "libklbheader_ref.so")
    if os.path.exists(ref):
        L = ctypes.CDLL(ref)
        out = ctypes.create_string_buffer(len(b) + 64)
        n = L.ref_header_bytes((ctypes.c_uint32 * 5)(*xyzct), 1, (ctypes.c_float * 5)(1, 1, 2.5, 1, 1),
                               (ctypes.c_uint32 * 5)(*bs), 1, md, 0x84, 13,
                               offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), ctypes.c_size_t(nb), out,
                               len(b) + 64)
        assert n == len(b) and out.raw[:n] == b
