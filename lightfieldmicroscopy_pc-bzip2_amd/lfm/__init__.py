"""ctypes binding of liblfm.so (the MI355X-native .lfm encoder / decoder).

This is the same C ABI a Matlab MEX, a JNI wrapper or any other FFI caller
binds (include/lfm/*.h); Python is only a test / bench harness here.

GPU entry points need a visible gfx950 device; they raise LfmError when the
library or the device is missing (there is no CPU fallback for the predictor
stage).  When PyTorch is importable it is imported BEFORE liblfm.so is loaded,
so both share one HIP runtime (libamdhip64.so.7) in the process.
"""
import ctypes
import os

import numpy as np

try:  # one HIP runtime per process: torch's, if torch is present
    import torch  # noqa: F401
    _HAVE_TORCH = True
except Exception:  # pragma: no cover
    _HAVE_TORCH = False

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("LFM_LIB") or os.path.join(PKG_DIR, "liblfm.so")

FAMILIES = {"tiles": 0, "angle_and_space": 0, "angle": 1, "space": 2}
DTYPES = {np.dtype(np.uint8): 0, np.dtype(np.uint16): 1, np.dtype(np.uint32): 2, np.dtype(np.uint64): 3,
          np.dtype(np.int8): 4, np.dtype(np.int16): 5, np.dtype(np.int32): 6, np.dtype(np.int64): 7,
          np.dtype(np.float32): 8, np.dtype(np.float64): 9}
NP_OF = {v: k for k, v in DTYPES.items()}

EXPORTS = [
    # klb_Cwrapper.h
    "writeKLBstack", "writeKLBstackSlices", "readKLBheader", "readKLBstack", "readKLBstackInPlace",
    "readKLBroiInPlace",
    # lfm_api.h
    "lfm_set_family", "lfm_get_family", "lfm_version", "lfm_api_version", "writeLFMstack_c", "readLFMstack_c",
    "lfm_encoder_create", "lfm_encoder_destroy", "lfm_encoder_encode", "lfm_encoder_encode_slab",
    "lfm_merge_slabs", "lfm_free", "lfm_decode_memory", "lfm_decode_memory_roi", "lfm_set_devices", "lfm_get_devices", "lfm_default_devices",
    "lfm_encoder_encode_multi", "lfm_release_encoders", "lfm_slab_info", "lfm_place_slab", "lfm_encoder_submit",
    "lfm_encoder_submit_select", "lfm_encoder_wait",
    # lfm_hip.h
    "lfm_hip_predict", "lfm_hip_unpredict", "lfm_hip_unpredict_async", "lfm_hip_unpredict_check",
    "lfm_hip_predict_candidates", "lfm_hip_entropy2d", "lfm_hip_select_workspace_bytes", "lfm_hip_select",
    "lfm_hip_synth", "lfm_hip_device_count", "lfm_hip_force_generic", "lfm_hip_bzip2_workspace_bytes",
    "lfm_hip_bzip2_blocks", "lfm_hip_bzip2_last_stage_ms", "lfm_hip_bunzip2_workspace_bytes", "lfm_hip_bunzip2_blocks", "lfm_hip_scatter_blocks",
]


class LfmError(RuntimeError):
    pass


class EncodeStats(ctypes.Structure):
    _fields_ = [("total_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double), ("select_ms", ctypes.c_double),
                ("predict_ms", ctypes.c_double), ("d2h_ms", ctypes.c_double), ("compress_ms", ctypes.c_double),
                ("chosen", ctypes.c_int), ("header_version", ctypes.c_int), ("entropy", ctypes.c_float * 8),
                ("out_bytes", ctypes.c_uint64), ("bz_stage_ms", ctypes.c_double * 5), ("bz_in_bytes", ctypes.c_uint64)]
    BZ_STAGES = ("rle1", "bwt", "mtf", "huffman", "emit")

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_ if f not in ("entropy", "bz_stage_ms")}
        d["entropy"] = list(self.entropy)
        d["bz_stage_ms"] = dict(zip(self.BZ_STAGES, list(self.bz_stage_ms)))
        return d


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LfmError("liblfm.so is not built (run `make -C %s` or __graft_entry__.build())" % PKG_DIR)
    L = ctypes.CDLL(LIB_PATH)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    f32p = ctypes.POINTER(ctypes.c_float)
    vp = ctypes.c_void_p
    L.writeKLBstack.argtypes = [vp, ctypes.c_char_p, u32p, ctypes.c_int, ctypes.c_int, f32p, u32p, ctypes.c_int,
                                ctypes.c_char_p]
    L.writeKLBstackSlices.argtypes = [ctypes.POINTER(vp), ctypes.c_char_p, u32p, ctypes.c_int, ctypes.c_int, f32p,
                                      u32p, ctypes.c_int, ctypes.c_char_p]
    L.readKLBheader.argtypes = [ctypes.c_char_p, u32p, ctypes.POINTER(ctypes.c_int), f32p, u32p,
                                ctypes.POINTER(ctypes.c_int), ctypes.c_char_p]
    L.readKLBstack.restype = vp
    L.readKLBstack.argtypes = [ctypes.c_char_p, u32p, ctypes.POINTER(ctypes.c_int), ctypes.c_int, f32p, u32p,
                               ctypes.POINTER(ctypes.c_int), ctypes.c_char_p]
    L.readKLBstackInPlace.argtypes = [ctypes.c_char_p, vp, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.readKLBroiInPlace.argtypes = [ctypes.c_char_p, vp, u32p, u32p, ctypes.c_int]
    L.lfm_version.restype = ctypes.c_char_p
    # lfm_decode_memory_roi's argument list (lfm_api.h); a library without the
    # version symbol is a round-5 build, whose list is the same
    if hasattr(L, "lfm_api_version") and L.lfm_api_version() != 2:
        raise OSError("liblfm.so API version %d, this binding needs 2" % L.lfm_api_version())
    L.writeLFMstack_c.argtypes = [vp, ctypes.c_char_p, u32p, ctypes.c_int, ctypes.c_int, f32p, u32p, ctypes.c_int,
                                  ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.readLFMstack_c.argtypes = [ctypes.c_char_p, vp, ctypes.c_int, ctypes.POINTER(ctypes.c_uint8),
                                 ctypes.POINTER(ctypes.c_uint8)]
    L.lfm_encoder_create.restype = vp
    L.lfm_encoder_create.argtypes = [ctypes.c_int, ctypes.c_int]
    L.lfm_encoder_destroy.argtypes = [vp]
    L.lfm_encoder_encode.argtypes = [vp, vp, ctypes.c_int, u32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, u32p,
                                     ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                     ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(EncodeStats)]
    L.lfm_encoder_encode_slab.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_uint32, u32p, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int, u32p, ctypes.c_int, ctypes.c_char_p,
                                          ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                          ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(EncodeStats)]
    L.lfm_encoder_submit.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_uint32, u32p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, u32p, ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_uint64)]
    L.lfm_encoder_submit_select.argtypes = [vp, vp, ctypes.c_int, vp, ctypes.c_uint32, vp, u32p, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, u32p, ctypes.c_int, ctypes.c_char_p,
                                            ctypes.POINTER(ctypes.c_uint64)]
    L.lfm_encoder_wait.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                   ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(EncodeStats)]
    L.lfm_encoder_encode_multi.argtypes = [vp, vp, u32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, u32p,
                                           ctypes.c_int, ctypes.c_char_p,
                                           ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)),
                                           ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(EncodeStats)]
    L.lfm_slab_info.argtypes = [vp, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.lfm_place_slab.argtypes = [vp, ctypes.c_uint64, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                 ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int]
    L.lfm_set_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.lfm_get_devices.argtypes = [ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.lfm_default_devices.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    L.lfm_release_encoders.argtypes = []
    L.lfm_release_encoders.restype = None
    L.lfm_merge_slabs.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_uint64), ctypes.c_int,
                                  ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(ctypes.c_uint64)]
    L.lfm_free.argtypes = [vp]
    L.lfm_free.restype = None
    L.lfm_decode_memory.argtypes = [ctypes.c_char_p, ctypes.c_uint64, vp, ctypes.c_int]
    L.lfm_decode_memory_roi.argtypes = [vp, ctypes.c_uint64, u32p, u32p, vp, ctypes.c_uint64, ctypes.c_int]
    L.lfm_hip_predict.argtypes = [vp, vp, vp] + [ctypes.c_int] * 8 + [vp]
    L.lfm_hip_unpredict.argtypes = [vp, vp, vp] + [ctypes.c_int] * 8 + [vp]
    L.lfm_hip_predict_candidates.argtypes = [vp, vp] + [ctypes.c_int] * 4 + [vp]
    L.lfm_hip_entropy2d.argtypes = [vp, ctypes.c_uint64, f32p, vp]
    L.lfm_hip_bzip2_workspace_bytes.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    L.lfm_hip_bzip2_workspace_bytes.restype = ctypes.c_size_t
    L.lfm_hip_bzip2_blocks.argtypes = [vp, u32p, u32p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                       ctypes.c_uint32, vp, ctypes.c_size_t, vp,
                                       ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32), vp]
    L.lfm_hip_bunzip2_workspace_bytes.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
    L.lfm_hip_bunzip2_workspace_bytes.restype = ctypes.c_size_t
    L.lfm_hip_bunzip2_blocks.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32, vp, ctypes.c_uint32,
                                         vp, ctypes.c_size_t, u32p, u32p, vp]
    L.lfm_hip_scatter_blocks.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, u32p, u32p,
                                         ctypes.c_uint32, vp, vp]
    L.lfm_hip_select_workspace_bytes.restype = ctypes.c_size_t
    L.lfm_hip_select_workspace_bytes.argtypes = [ctypes.c_int, ctypes.c_int]
    L.lfm_hip_select.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, f32p,
                                 ctypes.POINTER(ctypes.c_int), vp, vp]
    L.lfm_hip_synth.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, vp]
    _lib = L
    return L


def missing_exports():
    L = lib()
    return [name for name in EXPORTS if not hasattr(L, name)]


def device_count():
    return int(lib().lfm_hip_device_count())


def require_gpu():
    if device_count() <= 0:
        raise LfmError("no HIP device visible: the LFM predictor stage runs only on the GPU")


def set_devices(devices=None):
    """Devices the writers farm block ranges to (lfm_set_devices); None or []
    restores the default (see default_devices)."""
    devices = list(devices or [])
    arr = (ctypes.c_int * max(1, len(devices)))(*devices)
    _check(lib().lfm_set_devices(arr, len(devices)), "lfm_set_devices")


def get_devices():
    arr = (ctypes.c_int * 256)()
    n = lib().lfm_get_devices(arr, 256)
    return list(arr[:min(n, 256)])


def default_devices(n_visible, current=-1):
    """The writers' default device list on a machine with n_visible devices
    (lfm_default_devices: env LFM_GPUS / LOCAL_WORLD_SIZE / LOCAL_RANK / ...;
    no device call)."""
    arr = (ctypes.c_int * 256)()
    n = lib().lfm_default_devices(int(n_visible), int(current), arr, 256)
    return list(arr[:min(n, 256)])


def release_encoders():
    """Free the device / pinned buffers the writers keep between calls."""
    lib().lfm_release_encoders()


def set_family(family):
    if lib().lfm_set_family(FAMILIES.get(family, family)) != 0:
        raise LfmError("bad family %r" % (family,))


def get_family():
    return int(lib().lfm_get_family())


def _u32(v):
    return (ctypes.c_uint32 * 5)(*[int(x) for x in v])


def _f32(v):
    return (ctypes.c_float * 5)(*[float(x) for x in v])


def _xyzct(arr):
    a = arr
    while a.ndim < 5:
        a = a[None]
    t, c, z, y, x = a.shape
    return [x, y, z, c, t]


def _meta(m):
    if m is None:
        return None
    b = m.encode() if isinstance(m, str) else bytes(m)
    return ctypes.create_string_buffer(b[:256].ljust(256, b"\0"), 256)


def _check(rc, what):
    if rc != 0:
        raise LfmError("%s failed with code %d" % (what, rc))


# ------------------------------------------------------------- file API --
def write_lfm(path, img, predictor_request=0, nnum=13, video=0, block_size=None, pixel_size=None,
              compression=1, metadata=None, num_threads=-1, family=None):
    """MEX writeLFMstack semantics.  img: ndarray indexed [t, c, z, y, x] (or fewer leading dims)."""
    img = np.ascontiguousarray(img)
    if family is not None:
        set_family(family)
    xyzct = _xyzct(img)
    rc = lib().writeLFMstack_c(img.ctypes.data, os.fsencode(path), _u32(xyzct), DTYPES[img.dtype], num_threads,
                               _f32(pixel_size) if pixel_size is not None else None,
                               _u32(block_size) if block_size is not None else None, compression, _meta(metadata),
                               int(predictor_request), int(nnum), int(video))
    _check(rc, "writeLFMstack_c")


def write_klb(path, img, block_size=None, pixel_size=None, compression=1, metadata=None, num_threads=-1):
    """writeKLBstack (C ABI): headerVersion 0 (auto predictor), Nnum 13."""
    img = np.ascontiguousarray(img)
    rc = lib().writeKLBstack(img.ctypes.data, os.fsencode(path), _u32(_xyzct(img)), DTYPES[img.dtype], num_threads,
                             _f32(pixel_size) if pixel_size is not None else None,
                             _u32(block_size) if block_size is not None else None, compression, _meta(metadata))
    _check(rc, "writeKLBstack")


def read_header(path):
    xyzct = (ctypes.c_uint32 * 5)()
    dt = ctypes.c_int()
    ps = (ctypes.c_float * 5)()
    bs = (ctypes.c_uint32 * 5)()
    ct = ctypes.c_int()
    md = ctypes.create_string_buffer(256)
    _check(lib().readKLBheader(os.fsencode(path), xyzct, ctypes.byref(dt), ps, bs, ctypes.byref(ct), md),
           "readKLBheader")
    return dict(xyzct=list(xyzct), data_type=dt.value, pixel_size=list(ps), block_size=list(bs),
                compression=ct.value, metadata=md.raw)


def read_lfm(path, num_threads=-1, family=None):
    """Decode a .lfm file; returns (ndarray [t, c, z, y, x], header_version, nnum)."""
    if family is not None:
        set_family(family)
    h = read_header(path)
    x, y, z, c, t = h["xyzct"]
    out = np.empty((t, c, z, y, x), dtype=NP_OF[h["data_type"]])
    hv = ctypes.c_uint8()
    nn = ctypes.c_uint8()
    _check(lib().readLFMstack_c(os.fsencode(path), out.ctypes.data, num_threads, ctypes.byref(hv), ctypes.byref(nn)),
           "readLFMstack_c")
    return out, hv.value, nn.value


# ------------------------------------------------------ in-memory encoder --
class Encoder:
    """lfm_encoder: encode host arrays or device-resident tensors to .lfm bytes."""

    def __init__(self, device=-1, num_threads=-1):
        if device < 0 and _HAVE_TORCH and torch.cuda.is_available():
            device = torch.cuda.current_device()
        self._device = device
        self._h = lib().lfm_encoder_create(device, num_threads)
        if not self._h:
            raise LfmError("lfm_encoder_create failed")

    def close(self):
        if self._h:
            lib().lfm_encoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    _TORCH_KLB = {"torch.uint8": 0, "torch.uint16": 1, "torch.int16": 1, "torch.uint32": 2, "torch.uint64": 3,
                  "torch.int8": 4, "torch.int32": 6, "torch.int64": 7, "torch.float32": 8, "torch.float64": 9}

    def _operand(self, img, xyzct, data_type):
        """(pointer, is_device, xyzct, data_type, keepalive) of a numpy array or torch tensor.
        A CUDA tensor must be contiguous and live on this encoder's device;
        int16 is taken as a uint16 view (torch has no uint16 arithmetic)."""
        if _HAVE_TORCH and isinstance(img, torch.Tensor):
            if img.is_cuda:
                if not img.is_contiguous():
                    raise LfmError("device input must be contiguous (got strides %s)" % (img.stride(),))
                if self._device >= 0 and img.device.index != self._device:
                    raise LfmError("device input lives on cuda:%d, the encoder on cuda:%d"
                                   % (img.device.index, self._device))
                kt = self._TORCH_KLB.get(str(img.dtype))
                if kt is None:
                    raise LfmError("unsupported tensor dtype %s" % img.dtype)
                if data_type is not None and data_type != kt and not (data_type == 1 and kt in (1, 5)):
                    raise LfmError("data_type %d does not match tensor dtype %s" % (data_type, img.dtype))
                # the library orders its reads after the null stream's work
                # (torch's default stream); a producer on another current
                # stream is waited for here
                cur = torch.cuda.current_stream(img.device)
                if cur != torch.cuda.default_stream(img.device):
                    cur.synchronize()
                shape = list(img.shape)
                while len(shape) < 5:
                    shape = [1] + shape
                xyzct = xyzct or [shape[4], shape[3], shape[2], shape[1], shape[0]]
                return img.data_ptr(), 1, xyzct, (kt if data_type is None else data_type), img
            img = img.numpy()
        img = np.ascontiguousarray(img)
        xyzct = xyzct or _xyzct(img)
        data_type = DTYPES[img.dtype] if data_type is None else data_type
        return img.ctypes.data, 0, xyzct, data_type, img

    def encode(self, img, header_version=0, nnum=13, block_size=None, compression=1, metadata=None,
               xyzct=None, data_type=None, copy=True):
        """img: numpy array [t,c,z,y,x] (host) or a torch CUDA tensor (device, uint16 viewed as int16 ok).
        Returns (.lfm, stats dict): bytes, or with copy=False a zero-copy
        memoryview of the encoder's buffer, valid until its next call."""
        ptr, dev, xyzct, data_type, keep = self._operand(img, xyzct, data_type)
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_uint64()
        st = EncodeStats()
        rc = lib().lfm_encoder_encode(self._h, ptr, dev, _u32(xyzct), data_type, int(header_version), int(nnum),
                                      _u32(block_size) if block_size is not None else None, compression,
                                      _meta(metadata), ctypes.byref(out), ctypes.byref(n), ctypes.byref(st))
        _check(rc, "lfm_encoder_encode")
        del keep
        if not copy:
            return memoryview((ctypes.c_uint8 * n.value).from_address(ctypes.addressof(out.contents))), st.as_dict()
        return ctypes.string_at(out, n.value), st.as_dict()

    def submit(self, img, z0=0, prev=None, header_version=0, nnum=13, block_size=None, compression=1,
               metadata=None, xyzct=None, data_type=None, select_frame=None):
        """Pipelined encode (lfm_encoder_submit) of a stack (z0 = 0) or a z-slab:
        returns a ticket once every kernel has run (img may be released); the
        .lfm's last payload copies finish in the background.  wait(ticket)
        gives (.lfm, stats); at most two encodes are in flight.
        select_frame: the frame auto-selection runs on (the whole stack's frame
        0 for a slab; lfm_encoder_submit_select), same residency as img."""
        ptr, dev, xyzct, data_type, keep = self._operand(img, xyzct, data_type)
        pptr = None
        if prev is not None:
            pptr, pdev, _, _, pkeep = self._operand(prev, [1, 1, 1, 1, 1], data_type)
            if pdev != dev:
                raise LfmError("prev must live where img lives (host or device)")
        sptr = None
        if select_frame is not None:
            sptr, sdev, _, _, skeep = self._operand(select_frame, [1, 1, 1, 1, 1], data_type)
            if sdev != dev:
                raise LfmError("select_frame must live where img lives (host or device)")
        t = ctypes.c_uint64()
        rc = lib().lfm_encoder_submit_select(self._h, ptr, dev, pptr, int(z0), sptr, _u32(xyzct), data_type,
                                             int(header_version), int(nnum),
                                             _u32(block_size) if block_size is not None else None, compression,
                                             _meta(metadata), ctypes.byref(t))
        _check(rc, "lfm_encoder_submit_select")
        del keep
        return t.value

    def wait(self, ticket, copy=True):
        """(.lfm, stats) of a submitted encode; with copy=False a zero-copy
        memoryview valid until the second submit after it."""
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_uint64()
        st = EncodeStats()
        rc = lib().lfm_encoder_wait(self._h, ticket, ctypes.byref(out), ctypes.byref(n), ctypes.byref(st))
        _check(rc, "lfm_encoder_wait")
        if not copy:
            return memoryview((ctypes.c_uint8 * n.value).from_address(ctypes.addressof(out.contents))), st.as_dict()
        return ctypes.string_at(out, n.value), st.as_dict()

    def encode_multi(self, img, header_version=0, nnum=13, block_size=None, compression=1, metadata=None,
                     data_type=None, copy=True):
        """Encode a HOST stack on every device of set_devices() (the multi-GPU
        block scheduler behind klb_imageIO::writeImage).  Returns (.lfm, stats)."""
        img = np.ascontiguousarray(img)
        xyzct = _xyzct(img)
        data_type = DTYPES[img.dtype] if data_type is None else data_type
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_uint64()
        st = EncodeStats()
        rc = lib().lfm_encoder_encode_multi(self._h, img.ctypes.data, _u32(xyzct), data_type, int(header_version),
                                            int(nnum), _u32(block_size) if block_size is not None else None,
                                            compression, _meta(metadata), ctypes.byref(out), ctypes.byref(n),
                                            ctypes.byref(st))
        _check(rc, "lfm_encoder_encode_multi")
        if not copy:
            return memoryview((ctypes.c_uint8 * n.value).from_address(ctypes.addressof(out.contents))), st.as_dict()
        return ctypes.string_at(out, n.value), st.as_dict()

    def encode_slab(self, img, z0, prev=None, header_version=8, nnum=13, block_size=None, compression=1,
                    metadata=None, xyzct=None, data_type=None, copy=True):
        """Encode the z-slab of a larger stack that starts at global frame z0
        (see lfm_encoder_encode_slab); prev = raw frame z0-1 (same residency
        as img), needed when the slab starts at an odd frame of a video stack.
        Returns (slab .lfm bytes, stats)."""
        ptr, dev, xyzct, data_type, keep = self._operand(img, xyzct, data_type)
        pptr = None
        if prev is not None:
            pptr, pdev, _, _, pkeep = self._operand(prev, [1, 1, 1, 1, 1], data_type)
            if pdev != dev:
                raise LfmError("prev must live where img lives (host or device)")
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_uint64()
        st = EncodeStats()
        rc = lib().lfm_encoder_encode_slab(self._h, ptr, dev, pptr, int(z0), _u32(xyzct), data_type,
                                           int(header_version), int(nnum),
                                           _u32(block_size) if block_size is not None else None, compression,
                                           _meta(metadata), ctypes.byref(out), ctypes.byref(n), ctypes.byref(st))
        _check(rc, "lfm_encoder_encode_slab")
        del keep
        if not copy:
            return memoryview((ctypes.c_uint8 * n.value).from_address(ctypes.addressof(out.contents))), st.as_dict()
        return ctypes.string_at(out, n.value), st.as_dict()


def merge_slabs(slabs):
    """Join the .lfm bytes of consecutive z-slabs into the whole stack's .lfm."""
    n = len(slabs)
    arr = (ctypes.c_char_p * n)(*[bytes(b) for b in slabs])
    lens = (ctypes.c_uint64 * n)(*[len(b) for b in slabs])
    out = ctypes.POINTER(ctypes.c_uint8)()
    ln = ctypes.c_uint64()
    _check(lib().lfm_merge_slabs(arr, lens, n, ctypes.byref(out), ctypes.byref(ln)), "lfm_merge_slabs")
    try:
        return ctypes.string_at(out, ln.value)
    finally:
        lib().lfm_free(out)


def _addr(buf):
    """Address of a bytes / memoryview / numpy buffer (kept alive by the caller)."""
    if isinstance(buf, np.ndarray):
        return buf.ctypes.data
    if isinstance(buf, bytes):
        return ctypes.cast(ctypes.c_char_p(buf), ctypes.c_void_p).value
    return np.frombuffer(buf, dtype=np.uint8).ctypes.data


def slab_info(slab):
    """(payload bytes, block count) of a slab .lfm (what multi-process ranks exchange)."""
    pb, nb = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().lfm_slab_info(_addr(slab), len(slab), ctypes.byref(pb), ctypes.byref(nb)), "lfm_slab_info")
    return pb.value, nb.value


def place_slab(slab, dst, total_z, total_blocks, block_index, payload_offset, num_threads=-1):
    """Place one rank's z-slab .lfm into the whole stack's .lfm buffer `dst`
    (a writable numpy uint8 array, e.g. over shared memory) -- lfm_place_slab."""
    _check(lib().lfm_place_slab(_addr(slab), len(slab), dst.ctypes.data, dst.nbytes, int(total_z), int(total_blocks),
                                int(block_index), int(payload_offset), num_threads), "lfm_place_slab")


def decode(buf, shape_tczyx=None, dtype=np.uint16, num_threads=-1):
    if shape_tczyx is None:
        import struct
        xyzct = struct.unpack_from("<5I", buf, 2)
        dtype = NP_OF[int(np.frombuffer(buf, dtype=np.uint8, count=43)[42])]
        shape_tczyx = (xyzct[4], xyzct[3], xyzct[2], xyzct[1], xyzct[0])
    out = np.empty(shape_tczyx, dtype=dtype)
    _check(lib().lfm_decode_memory(buf, len(buf), out.ctypes.data, num_threads), "lfm_decode_memory")
    return out


def decode_roi(buf, lb, ub, dtype=None, num_threads=-1, out=None):
    """Region lb .. ub (inclusive, [x, y, z, c, t]) of an in-memory .lfm
    (lfm_decode_memory_roi); returns an array [t, c, z, y, x] of the region in
    the file's data type (header byte 42).  `dtype`, when given, must be that
    type.  `out` (optional): a C-contiguous array of the region's size and the
    file's dtype to decode into (readKLBroiInPlace's caller-owned buffer),
    returned reshaped.  The library checks the byte count as well."""
    if len(buf) < 43:
        raise ValueError("decode_roi: %d bytes hold no .lfm header" % len(buf))
    dt = int(np.frombuffer(buf, dtype=np.uint8, count=43)[42])  # (buf may be bytes, a numpy array or a memoryview)
    if dt not in NP_OF:
        raise ValueError("decode_roi: unknown data type %d in the header" % dt)
    fdt = np.dtype(NP_OF[dt])
    if dtype is not None and np.dtype(dtype) != fdt:
        raise ValueError("decode_roi: the file holds %s, not %s" % (fdt, np.dtype(dtype)))
    shape = tuple(int(u) - int(l) + 1 for l, u in zip(lb, ub))[::-1]
    if out is None:
        out = np.empty(shape, dtype=fdt)
    else:
        if not isinstance(out, np.ndarray) or not out.flags.c_contiguous or not out.flags.writeable:
            raise ValueError("decode_roi: out must be a writeable C-contiguous numpy array")
        if out.dtype != fdt or out.size != int(np.prod(shape)):
            raise ValueError("decode_roi: out holds %d x %s, the region is %s x %s" % (out.size, out.dtype, shape, fdt))
        out = out.reshape(shape)
    _check(lib().lfm_decode_memory_roi(_addr(buf), len(buf), _u32(lb), _u32(ub), out.ctypes.data, out.nbytes,
                                       num_threads), "lfm_decode_memory_roi")
    return out


# ------------------------------------------------------ device primitives --
def _stream(stream):
    if stream is None:
        return None
    return ctypes.c_void_p(int(stream.cuda_stream) if hasattr(stream, "cuda_stream") else int(stream))


def predict_device(d_in, d_out, W, H, nframes, T, family, predictor, video=0, z0=0, d_prev=None, stream=None):
    """Launch the fused predictor + symbolize kernel on device tensors (or raw pointers)."""
    p = lambda t: None if t is None else (t.data_ptr() if hasattr(t, "data_ptr") else int(t))  # noqa: E731
    rc = lib().lfm_hip_predict(p(d_in), p(d_prev), p(d_out), W, H, nframes, T, FAMILIES.get(family, family),
                               predictor, video, z0, _stream(stream))
    _check(rc, "lfm_hip_predict")


def unpredict_device(d_sym, d_out, W, H, nframes, T, family, predictor, video=0, z0=0, d_prev=None, stream=None):
    """Inverse predictor (decode) on device tensors: symbols -> pixels."""
    p = lambda t: None if t is None else (t.data_ptr() if hasattr(t, "data_ptr") else int(t))  # noqa: E731
    rc = lib().lfm_hip_unpredict(p(d_sym), p(d_prev), p(d_out), W, H, nframes, T, FAMILIES.get(family, family),
                                 predictor, video, z0, _stream(stream))
    _check(rc, "lfm_hip_unpredict")


def predict_candidates_device(d_frame, d_out7, W, H, T, family, stream=None):
    """The seven spatial candidates of one frame in one launch (d_out7: 7*H*W uint16)."""
    rc = lib().lfm_hip_predict_candidates(d_frame.data_ptr(), d_out7.data_ptr(), W, H, T,
                                          FAMILIES.get(family, family), _stream(stream))
    _check(rc, "lfm_hip_predict_candidates")


def select_device(d_frame, W, H, T, family, stream=None):
    ent = (ctypes.c_float * 8)()
    k = ctypes.c_int()
    rc = lib().lfm_hip_select(d_frame.data_ptr(), W, H, T, FAMILIES.get(family, family), ent, ctypes.byref(k), None,
                              _stream(stream))
    _check(rc, "lfm_hip_select")
    return k.value, np.array(list(ent), dtype=np.float32)


def entropy_device(d_cand, npix=None, stream=None):
    e = ctypes.c_float()
    n = d_cand.numel() if npix is None else npix
    _check(lib().lfm_hip_entropy2d(d_cand.data_ptr(), n, ctypes.byref(e), _stream(stream)), "lfm_hip_entropy2d")
    return e.value


def bzip2_device(d_img, dims, block, bpp, level=None, first=0, count=None, stream=None):
    """GPU bzip2 of the x-fastest block grid of a device image (torch tensor
    holding dims[4]*...*dims[0]*bpp bytes).  Returns ([bytes or None per
    stream], flags): None where the stream was handed to the host library."""
    nb = [-(-d // b) for d, b in zip(dims, block)]
    total = int(np.prod(nb))
    count = total - first if count is None else count
    block_bytes = int(np.prod(block)) * bpp
    level = min(9, -(-block_bytes // 100000)) if level is None else level
    ws_bytes = lib().lfm_hip_bzip2_workspace_bytes(count, block_bytes)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=d_img.device)
    out_cap = ((block_bytes + block_bytes // 50 + 4096 + 255) // 256) * 256
    pay = torch.empty(count * out_cap, dtype=torch.uint8, device=d_img.device)
    sizes = (ctypes.c_uint64 * count)()
    flags = (ctypes.c_uint32 * count)()
    _check(lib().lfm_hip_bzip2_blocks(d_img.data_ptr(), _u32(dims), _u32(block), bpp, first, count, level,
                                      ws.data_ptr(), ws_bytes, pay.data_ptr(), sizes, flags, _stream(stream)),
           "lfm_hip_bzip2_blocks")
    host = pay[:int(sum(sizes))].cpu().numpy().tobytes()
    out, o = [], 0
    for i in range(count):
        if flags[i]:
            out.append(None)
        else:
            out.append(host[o:o + sizes[i]])
            o += sizes[i]
    return out, list(flags)


def bunzip2_device(streams, out_stride, device="cuda", stream=None):
    """GPU bzip2 decode of single-block streams (bytes objects).  Returns
    ([bytes per stream, or None where the device flagged it for the host
    library], flags): flag 1 = host library, 2 = block CRC mismatch."""
    count = len(streams)
    offs = np.zeros(count + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(x) for x in streams])
    blob = b"".join(streams) + bytes(64)
    d_pay = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(device)
    ws_bytes = lib().lfm_hip_bunzip2_workspace_bytes(count, out_stride)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=device)
    out = torch.empty(count * out_stride, dtype=torch.uint8, device=device)
    lens = (ctypes.c_uint32 * count)()
    flags = (ctypes.c_uint32 * count)()
    _check(lib().lfm_hip_bunzip2_blocks(d_pay.data_ptr(), offs.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), count,
                                        out.data_ptr(), out_stride, ws.data_ptr(), ws_bytes, lens, flags,
                                        _stream(stream)), "lfm_hip_bunzip2_blocks")
    host = out.cpu().numpy()
    res = [None if flags[i] else host[i * out_stride:i * out_stride + lens[i]].tobytes() for i in range(count)]
    return res, list(flags)


def synth_device(d_out, X, Y, Z, T, t_index=0, idx0=None, seed=0x4C464D00, z0=0, stream=None):
    """SURVEY 8(d) generator on the device: frames z0 .. z0+Z-1 of volume
    (0, t_index); idx0 defaults to z0*X*Y (a z-slab of a c = t = 1 stack,
    equal to oracle.synthetic_lf(..., z0=z0))."""
    if idx0 is None:
        idx0 = z0 * X * Y
    _check(lib().lfm_hip_synth(d_out.data_ptr(), X, Y, Z, T, t_index, z0, idx0, seed, _stream(stream)),
           "lfm_hip_synth")
