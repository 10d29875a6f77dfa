"""CPU oracle for the .lfm encode/decode path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module; the product never does.

Pixel arithmetic lives in lfm_oracle.c (ctypes); this module restates the
container around it:
  * header bytes           klb_imageHeader.cpp:164-176 (FILE* writeHeader)
  * block decomposition    klb_imageIO.cpp:98-160 (x-fastest block ids,
                           border blocks clipped, gather x-fastest)
  * bzip2 level            klb_imageIO.cpp:108 (min(9, ceil(blockBytes/1e5)),
                           blockBytes = nominal block after the clamp at :2402-2404)
  * bzip2 call             klb_imageIO.cpp:217 (BZ2_bzBuffToBuffCompress,
                           verbosity 0, workFactor 30)
  * in-order writer        klb_imageIO.cpp:1145-1225 (blockOffset = cumulative
                           END offsets, rewritten after the blocks)
  * predictor stage        klb_imageIO.cpp:2271-2399 (auto-select on frame 0
                           when request < 8; forced request-8 via & 0x77)
bzip2 comes from oracle/_ref/libbz2_ref.so (the reference's vendored
bzip2-1.0.6 compiled from its own sources) when present, else from Python's
bz2 module (system libbz2 1.0.8; byte-identical on the reference KATs).

Divergences from the reference, decided in SURVEY.md section 8(a) and kept
identical in the product: for c*t > 1 every (c,t) volume runs its own z loop
(the reference leaves those frames zero), selection uses frame (z=0,c=0,t=0)
only, requests >= 16 are rejected instead of writing an all-zero payload.
"""
import bz2 as _pybz2
import ctypes
import math
import os
import struct

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
FAMILY = {"tiles": 0, "angle_and_space": 0, "angle": 1, "space": 2}
BYTES_PER_PIXEL = {0: 1, 1: 2, 2: 4, 3: 8, 4: 1, 5: 2, 6: 4, 7: 8, 8: 4, 9: 8}
HEADER_FIXED = 320

_lib = None
_bz = None


def lib():
    global _lib
    if _lib is None:
        p = os.path.join(HERE, "liblfm_oracle.so")
        if not os.path.exists(p):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = ctypes.CDLL(p)
        u16p = ctypes.POINTER(ctypes.c_uint16)
        L.lfmo_predict_frame.argtypes = [u16p, u16p, u16p] + [ctypes.c_int] * 6
        L.lfmo_predict_volume.argtypes = [u16p, u16p] + [ctypes.c_int] * 7
        L.lfmo_unpredict_volume.argtypes = [u16p, u16p] + [ctypes.c_int] * 7
        L.lfmo_unpredict_volume.restype = ctypes.c_int
        L.lfmo_unpredict_frame.argtypes = [u16p, u16p, u16p] + [ctypes.c_int] * 6
        L.lfmo_unpredict_frame.restype = ctypes.c_int
        L.lfmo_entropy2d.argtypes = [u16p, ctypes.c_uint64]
        L.lfmo_entropy2d.restype = ctypes.c_float
        L.lfmo_select.argtypes = [u16p] + [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_float)]
        L.lfmo_select.restype = ctypes.c_int
        L.lfmo_residual.argtypes = [u16p, u16p] + [ctypes.c_int] * 8
        L.lfmo_residual.restype = ctypes.c_int
        _lib = L
    return _lib


def _p16(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16))


# ----------------------------------------------------------------- bzip2 --
class _RefBz2:
    def __init__(self, path):
        self.L = ctypes.CDLL(path)
        self.L.BZ2_bzBuffToBuffCompress.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint),
                                                    ctypes.c_char_p, ctypes.c_uint,
                                                    ctypes.c_int, ctypes.c_int, ctypes.c_int]
        self.L.BZ2_bzBuffToBuffDecompress.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint),
                                                      ctypes.c_char_p, ctypes.c_uint,
                                                      ctypes.c_int, ctypes.c_int]
        self.kind = "reference bzip2-1.0.6 (oracle/_ref)"

    def compress(self, data, level, cap=None):
        cap = cap or int(math.ceil(len(data) * 2.0 + 50.0))
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_uint(cap)
        rc = self.L.BZ2_bzBuffToBuffCompress(out, ctypes.byref(n), data, len(data), level, 0, 30)
        if rc != 0:
            raise RuntimeError("BZ2_bzBuffToBuffCompress rc=%d" % rc)
        return out.raw[:n.value]

    def decompress(self, data, size):
        out = ctypes.create_string_buffer(size)
        n = ctypes.c_uint(size)
        rc = self.L.BZ2_bzBuffToBuffDecompress(out, ctypes.byref(n), data, len(data), 0, 0)
        if rc != 0:
            raise RuntimeError("BZ2_bzBuffToBuffDecompress rc=%d" % rc)
        return out.raw[:n.value]


class _PyBz2:
    kind = "python bz2 (system libbz2)"

    def compress(self, data, level, cap=None):
        return _pybz2.compress(data, level)

    def decompress(self, data, size):
        return _pybz2.decompress(data)


def bzip2():
    global _bz
    if _bz is None:
        p = os.path.join(HERE, "_ref", "libbz2_ref.so")
        _bz = _RefBz2(p) if os.path.exists(p) else _PyBz2()
    return _bz


# -------------------------------------------------------------- predictors --
def predict_frame(cur, prev, T, family, k, zflag):
    cur = np.ascontiguousarray(cur, dtype=np.uint16)
    H, W = cur.shape
    out = np.empty_like(cur)
    pv = np.ascontiguousarray(prev, dtype=np.uint16) if prev is not None else cur
    lib().lfmo_predict_frame(_p16(cur), _p16(pv), _p16(out), W, H, T, FAMILY.get(family, family), k, zflag)
    return out


def predict_volume(vol, T, family, k, video):
    """vol: (Z, H, W) uint16 -> symbols (Z, H, W) (Predictor_both semantics)."""
    vol = np.ascontiguousarray(vol, dtype=np.uint16)
    Z, H, W = vol.shape
    out = np.empty_like(vol)
    lib().lfmo_predict_volume(_p16(vol), _p16(out), W, H, Z, T, FAMILY.get(family, family), k, int(video))
    return out


def unpredict_volume(sym, T, family, k, video):
    sym = np.ascontiguousarray(sym, dtype=np.uint16)
    Z, H, W = sym.shape
    out = np.empty_like(sym)
    rc = lib().lfmo_unpredict_volume(_p16(sym), _p16(out), W, H, Z, T, FAMILY.get(family, family), k, int(video))
    if rc != 0:
        raise ValueError("temporal frames of the angle/space families are not invertible")
    return out


def entropy2d(cand):
    cand = np.ascontiguousarray(cand, dtype=np.uint16).ravel()
    return float(lib().lfmo_entropy2d(_p16(cand), cand.size))


def select(frame, T, family):
    frame = np.ascontiguousarray(frame, dtype=np.uint16)
    H, W = frame.shape
    ent = (ctypes.c_float * 8)()
    k = lib().lfmo_select(_p16(frame), W, H, T, FAMILY.get(family, family), ent)
    return k, np.array(list(ent), dtype=np.float32)


def predictor_stage(img, header_version, T, family, z0=0, prev=None):
    """img: (t, c, z, y, x) uint16.  Returns (symbols, header_version_out, entropies|None).

    klb_imageIO.cpp:2271-2399 with the per-volume decision for c*t > 1.
    z0 / prev: the stack is the z-slab starting at global frame z0 (c = t = 1)
    and prev is raw frame z0 - 1 (multi-GPU sharding)."""
    hv = int(header_version)
    req = hv & 0x7F
    video = (hv >> 7) & 1
    ent = None
    if req < 8:
        k, ent = select(img[0, 0, 0], T, family)
        hv_out = (hv & 0x80) | k
    else:
        k = hv & 0x77            # `headerVersion & 0x7F - 8` (precedence) = & 0x77
        if k > 7:
            raise ValueError("predictor request %d is not a valid forced request" % req)
        hv_out = (hv & 0x80) | k
    sym = np.empty_like(img)
    if z0:
        assert img.shape[0] == 1 and img.shape[1] == 1
        vol = img[0, 0]
        for z in range(vol.shape[0]):
            zf = (video & (z0 + z)) & 1
            p = vol[z - 1] if z else prev
            sym[0, 0, z] = predict_frame(vol[z], p if zf else None, T, family, k, zf) if k else vol[z]
        return sym, hv_out, ent
    for t in range(img.shape[0]):
        for c in range(img.shape[1]):
            sym[t, c] = predict_volume(img[t, c], T, family, k, video)
    return sym, hv_out, ent


# --------------------------------------------------------------- container --
def num_blocks_per_dim(xyzct, bs):
    # klb_imageHeader.cpp calculateNumBlocks: ceil((float)xyzct / (float)blockSize)
    return [int(math.ceil(np.float32(x) / np.float32(b))) for x, b in zip(xyzct, bs)]


def default_block_size(data_type):
    bpp = BYTES_PER_PIXEL[data_type]
    return [max(v // bpp, 1) for v in (192, 192, 16, 1, 1)]


def header_bytes(hv, nnum, xyzct, pixel_size, data_type, compression, metadata, block_size, offsets):
    b = struct.pack("<BB", hv & 0xFF, nnum & 0xFF)
    b += struct.pack("<5I", *xyzct) + struct.pack("<5f", *pixel_size)
    b += struct.pack("<BB", data_type, compression)
    md = bytes(metadata or b"")[:256]
    b += md + b"\0" * (256 - len(md))
    b += struct.pack("<5I", *block_size)
    b += np.asarray(offsets, dtype="<u8").tobytes()
    return b


def iter_blocks(xyzct, bs):
    nb = num_blocks_per_dim(xyzct, bs)
    total = int(np.prod(nb))
    for bid in range(total):
        rem = bid
        coord = []
        for d in range(5):
            coord.append((rem % nb[d]) * bs[d])
            rem //= nb[d]
        size = [min(bs[d], xyzct[d] - coord[d]) for d in range(5)]
        yield bid, coord, size


def gather_block(arr5, coord, size):
    """arr5 indexed [t, c, z, y, x]; returns the block's bytes, x fastest."""
    x0, y0, z0, c0, t0 = coord
    sx, sy, sz, sc, st = size
    return np.ascontiguousarray(arr5[t0:t0 + st, c0:c0 + sc, z0:z0 + sz, y0:y0 + sy, x0:x0 + sx]).tobytes()


def encode(img, header_version=0, nnum=13, family="tiles", block_size=None, pixel_size=None,
           metadata=None, compression=1, data_type=1, z0=0, prev=None):
    """img: ndarray shaped (t, c, z, y, x) (or fewer leading dims).  Returns .lfm bytes.
    z0 / prev: encode the z-slab starting at global frame z0 (see predictor_stage)."""
    img = np.asarray(img)
    while img.ndim < 5:
        img = img[None]
    xyzct = [img.shape[4], img.shape[3], img.shape[2], img.shape[1], img.shape[0]]
    bpp = BYTES_PER_PIXEL[data_type]
    bs = list(block_size) if block_size is not None else default_block_size(data_type)
    bs = [min(b, x) for b, x in zip(bs, xyzct)]                       # :2402-2404
    ps = list(pixel_size) if pixel_size is not None else [1.0] * 5
    if bpp == 2 and compression in (0, 1, 2):
        sym, hv, _ = predictor_stage(img.view(np.uint16), header_version, nnum, family, z0, prev)
    else:
        sym, hv = img, header_version & 0x80
    block_bytes = bpp * int(np.prod(bs))
    level = min(9, -(-block_bytes // 100000))                            # :108
    cap = int(math.ceil(float(np.float32(block_bytes) * np.float32(2.0) + np.float32(50.0))))
    blobs = []
    for _, coord, size in iter_blocks(xyzct, bs):
        raw = gather_block(sym, coord, size)
        if compression == 1:
            blobs.append(bzip2().compress(raw, level, cap))
        elif compression == 0:
            blobs.append(raw)
        else:
            raise NotImplementedError("oracle covers NONE and BZIP2 only")
    offsets = np.cumsum([len(b) for b in blobs]).astype(np.uint64)
    head = header_bytes(hv, nnum, xyzct, ps, data_type, compression, metadata, bs, offsets)
    return head + b"".join(blobs)


def parse_header(buf):
    hv, nnum = struct.unpack_from("<BB", buf, 0)
    xyzct = list(struct.unpack_from("<5I", buf, 2))
    ps = list(struct.unpack_from("<5f", buf, 22))
    dt, ct = struct.unpack_from("<BB", buf, 42)
    md = bytes(buf[44:300])
    bs = list(struct.unpack_from("<5I", buf, 300))
    nb = int(np.prod(num_blocks_per_dim(xyzct, bs)))
    offs = np.frombuffer(bytes(buf[320:320 + 8 * nb]), dtype="<u8")
    return dict(header_version=hv, nnum=nnum, xyzct=xyzct, pixel_size=ps, data_type=dt,
                compression=ct, metadata=md, block_size=bs, offsets=offs, nb=nb,
                header_size=320 + 8 * nb)


def decode(buf, family="tiles"):
    """Returns (img (t,c,z,y,x), header dict).  The predictor family is not
    stored in the file (compile-time LFM_PREDICTOR_WAY), so it is a parameter."""
    h = parse_header(buf)
    xyzct, bs = h["xyzct"], h["block_size"]
    bpp = BYTES_PER_PIXEL[h["data_type"]]
    dt = np.dtype("u%d" % bpp) if bpp in (1, 2, 4, 8) else np.uint8
    sym = np.zeros((xyzct[4], xyzct[3], xyzct[2], xyzct[1], xyzct[0]), dtype=dt)
    start = h["header_size"]
    prev = 0
    for bid, coord, size in iter_blocks(xyzct, bs):
        end = int(h["offsets"][bid])
        blob = bytes(buf[start + prev:start + end])
        nbytes = bpp * int(np.prod(size))
        raw = bzip2().decompress(blob, nbytes) if h["compression"] == 1 else blob
        x0, y0, z0, c0, t0 = coord
        sx, sy, sz, sc, st = size
        sym[t0:t0 + st, c0:c0 + sc, z0:z0 + sz, y0:y0 + sy, x0:x0 + sx] = \
            np.frombuffer(raw, dtype=dt).reshape(st, sc, sz, sy, sx)
        prev = end
    k = h["header_version"] & 0x7F
    video = h["header_version"] >> 7
    if bpp != 2 or k == 0:
        return sym, h
    out = np.empty_like(sym)
    for t in range(sym.shape[0]):
        for c in range(sym.shape[1]):
            out[t, c] = unpredict_volume(sym[t, c], h["nnum"], family, k, video)
    return out, h


# ------------------------------------------------------ synthetic inputs --
def splitmix64(x):
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def synthetic_lf(X, Y, Z=1, C=1, Tn=1, T=15, seed=0x4C464D00, z0=0, t0=0, idx0=None):
    """SURVEY.md section 8(d) integer light-field generator (numpy restatement).
    z0 > 0 (C = Tn = 1): frames [z0, z0 + Z) of a taller stack, so large
    stacks can be generated slab by slab.  t0 / idx0 (C = Tn = 1): frames of
    t-volume t0 of a larger 5-D stack whose linear index starts at idx0 (for
    frames z0.. of volume t0 of an X x Y x Zv x 1 x Tn stack:
    idx0 = (t0 * Zv + z0) * X * Y), so multi-volume stacks can be generated
    one volume (or slab) at a time."""
    if z0 or t0 or idx0 is not None:
        assert C == 1 and Tn == 1
    x = np.arange(X, dtype=np.int64)[None, None, None, None, :]
    y = np.arange(Y, dtype=np.int64)[None, None, None, :, None]
    z = np.arange(z0, z0 + Z, dtype=np.int64)[None, None, :, None, None]
    t = np.arange(t0, t0 + Tn, dtype=np.int64)[:, None, None, None, None]
    du = (x % T) - T // 2
    dv = (y % T) - T // 2
    r2 = du * du + dv * dv
    rm = 2 * (T // 2) * (T // 2) + 1
    lens = (1024 * (rm - r2)) // rm

    def tri(a):
        return np.abs((a % 2048) - 1024)
    field = 256 + tri(3 * x + 40 * z + 97 * t) // 4 + tri(2 * y) // 4
    shape = (Tn, C, Z, Y, X)
    i0 = z0 * Y * X if idx0 is None else int(idx0)
    idx = np.arange(i0, i0 + int(np.prod(shape)), dtype=np.uint64).reshape(shape)
    noise = (_splitmix_vec(np.uint64(seed) ^ (idx * np.uint64(0x9E3779B97F4A7C15))) >> np.uint64(58)).astype(np.int64)
    v = 100 + (lens * field) // 256 + noise
    return np.broadcast_to(v, shape).astype(np.uint16)


def _splitmix_vec(x):
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        z = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))
