"""Benchmark: uint16 Mpixel/s encode (predictor -> bzip2) on MI355X.

One step = encode one synthetic light-field stack of the BASELINE config 3 shape
(2048 x 2048 x 64 uint16, Nnum 15, angle family, predictor auto-selected on
frame 0) from HBM-resident input to a complete in-memory .lfm: GPU selection
(8 candidates, 2D entropy) + fused predictor/symbolize kernel over all 64 frames
+ GPU bzip2 of the 3 872 96x96x8 blocks (byte-identical to libbzip2) + D2H of
the compressed blocks into the pinned .lfm buffer, in order.  Nothing is cached
between steps.  After the timed steps (N=1) the last .lfm is decoded once
(GPU bzip2 decode + GPU inverse predictor) and compared with the input: `decode`
in the JSON line, for information (not the metric).

Multi-GPU (torchrun, one process per GPU): rank r encodes z-slab r (frames
64r .. 64r+63) of a (world x 64)-frame stack; every rank's submit selects the
predictor on the stack's frame 0 (handed in as select_frame, redundantly on
every rank: no broadcast) on the encoder's stream.  Inside the timed region the ranks then build ONE .lfm of the whole
stack in host shared memory: an all_gather of every slab's (payload bytes,
block count) -- the path's only exchange, RCCL under nccl -- gives each rank
its payload offset and first block index, and every rank places its own
compressed blocks and offset-table entries there concurrently
(lfm.place_slab; equal to lfm.merge_slabs).  Scaling "weak"; a barrier +
MAX-over-ranks of the timed region gives value.

After the timed steps the last .lfm is checked against the oracle's digests
(tests/golden/full_size_manifest.json, reference bzip2-1.0.6): the whole-file
SHA-256 of config 3 at N = 1, per-layer digests of the 512-frame stack at
N > 1 (`verified` in the JSON line).  At N = 1 the same stack is also encoded
from host memory (pinned and pageable), H2D inside the timed region:
`host_input` (the PCIe-inclusive rate; `value` is always HBM-resident).

At N = 1 more legs follow (not the metric): `configs_1_2` -- BASELINE
configs 1 (img.tif, predictor off; beside the reference's own CPU path) and 2
(512 x 512 space frame), bytes checked; `config5` -- four full
t-volumes of config 5 (4096 x 4096 x 32 x 1 x 4, video, tiles) encoded from
HBM into one .lfm (SHA-256 checked) and decoded back, the per-GPU rate of the
config-5 round trip; `inproc` -- the drop-in multi-GPU writer
(lfm_encoder_encode_multi, what klb_imageIO::writeImage / writeKLBstack run)
on config 4 from host memory, on this device and on every visible device.

Also reported: `roofline` of the dominant kernel (fused predictor, HIP-event
time per launch on its own stream) and `cpu_baseline` = the reference's CPU
bzip2-only path (request 8, same blocks, the reference's own bzip2-1.0.6 from
oracle/_ref) on a bounded sample, timed on this host.
"""
import argparse
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lightfieldmicroscopy_pc-bzip2_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402  (before liblfm: one HIP runtime)
import torch.distributed as dist  # noqa: E402

import lfm  # noqa: E402
from lfm.shard import max_over_ranks  # noqa: E402

X, Y, Z, T = 2048, 2048, 64, 15
FAMILY = "angle"
PEAK_HBM_GBS = 8000.0
SEED = 0x4C464D03


def host_threads(local_world):
    """bzip2 worker threads per rank: LFM_NUM_THREADS, else this process's CPU
    share (affinity, capped by OMP_NUM_THREADS, split across local ranks)."""
    v = os.environ.get("LFM_NUM_THREADS")
    if v and v.isdigit() and int(v) > 0:
        return int(v)
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    elif local_world > 1:
        n = n // local_world
    return max(1, n)


def cpu_baseline(seconds_budget=20.0, threads=None):
    """Reference CPU bzip2-only path (predictor off = request 8, default blocks)
    on a bounded z-slab of the same synthetic stack, with the reference's own
    bzip2 (oracle/_ref) on `threads` host threads."""
    import ctypes
    from concurrent.futures import ThreadPoolExecutor
    import lfm_oracle as O
    bz = O.bzip2()
    zs = 16
    img = O.synthetic_lf(X, Y, Z=zs, T=T, seed=SEED)
    xyzct = [X, Y, zs, 1, 1]
    bs = [96, 96, 8, 1, 1]
    blocks = list(O.iter_blocks(xyzct, bs))
    level = 2

    def one(b):
        _, coord, size = b
        return len(bz.compress(O.gather_block(img, coord, size), level))

    threads = threads or len(os.sched_getaffinity(0))
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        total = sum(ex.map(one, blocks))
    dt = time.perf_counter() - t0
    px = X * Y * zs
    # single-thread rate on a few blocks for context
    t1 = time.perf_counter()
    nb1 = 0
    for b in blocks[:24]:
        one(b)
        nb1 += 1
    dt1 = time.perf_counter() - t1
    px1 = nb1 * 96 * 96 * 8
    # BASELINE config 1 on the reference's CPU path: img.tif page 0 and the
    # 29-page stack, request 8, one thread, the reference's bzip2 (as above)
    tif = np.load(os.path.join(REPO, "tests", "golden", "img_tif.npz"))["img"]
    cfg1 = {}
    for name, im in (("page0", tif[0][None, None, None]), ("stack29", tif[None, None])):
        reps = 20
        t2 = time.perf_counter()
        for _ in range(reps):
            rb = O.encode(im, header_version=8, nnum=13, family="tiles")
        ms = (time.perf_counter() - t2) * 1e3 / reps
        px_i = int(np.prod(im.shape))
        cfg1[name] = {"Mpixel_per_s": round(px_i / ms / 1e3, 2), "ms": round(ms, 3),
                      "ratio": round(px_i * 2 / len(rb), 4)}
    return {"value": px / dt / 1e6, "unit": "Mpixel/s", "cores": threads, "config1": cfg1,
            "kind": "reference" if "reference" in bz.kind else "port",
            "sample": "%dx%dx%d uint16 synthetic slab of the bench stack, request 8 (predictor off), 96x96x8 blocks, "
                      "bzip2 level 2 (%s), %d blocks, ratio %.3f" % (X, Y, zs, bz.kind, len(blocks),
                                                                      px * 2 / total),
            "value_1thread": px1 / dt1 / 1e6, "nproc": os.cpu_count()}


def _manifest(name):
    path = os.path.join(REPO, "tests", "golden", "full_size_manifest.json")
    try:
        return {e["name"]: e for e in json.load(open(path))}.get(name)
    except (OSError, ValueError):
        return None


def verify_lfm(buf, world, zf):
    """Compare the timed .lfm with the oracle's digests (outside the timed region)."""
    if world == 1 and zf == Z:
        e = _manifest("cfg3_2048x2048x64_angle_auto")
        if e is None:
            return None
        return {"against": "cfg3 whole-file SHA-256 (oracle, reference bzip2-1.0.6)",
                "ok": hashlib.sha256(buf).hexdigest() == e["sha256"] and len(buf) == e["size"]}
    e = _manifest("cfg3x8_2048x2048x512_angle_auto")
    nlay = world * zf // 8
    if e is None or zf % 8 or nlay > len(e["layer_sha256"]):
        return None
    per = e["nblocks"] // len(e["layer_sha256"])
    nb = per * nlay
    offs = np.frombuffer(buf, dtype="<u8", count=nb, offset=320)
    base = 320 + 8 * nb
    ok = int(np.frombuffer(buf, dtype="<u4", count=5, offset=2)[2]) == world * zf
    prev = 0
    for j in range(nlay):
        end = int(offs[(j + 1) * per - 1])
        ok = ok and hashlib.sha256(buf[base + prev:base + end]).hexdigest() == e["layer_sha256"][j]
        prev = end
    ok = ok and len(buf) == base + prev
    if nlay == len(e["layer_sha256"]):
        ok = ok and hashlib.sha256(buf).hexdigest() == e["sha256"]
    return {"against": "%d layer SHA-256s of the %d-frame stack (oracle, reference bzip2-1.0.6)"
                       % (nlay, len(e["layer_sha256"]) * 8), "ok": bool(ok)}


def _free_bytes(d):
    try:
        st = os.statvfs(d)
        return st.f_bavail * st.f_frsize
    except OSError:
        return 0


class SharedLfm:
    """The whole stack's .lfm in host shared memory, written by every rank.
    The file is sparse: writes beyond the filesystem's free space would fault
    (SIGBUS on the mapping), so /dev/shm is used only when it can hold the
    whole capacity, else /tmp (same check), else the run stops with a message."""

    def __init__(self, rank, world, cap):
        port = os.environ.get("MASTER_PORT", "0")
        need = int(cap * 1.02) + (64 << 20)
        d = None
        for cand in ("/dev/shm", os.environ.get("TMPDIR", "/tmp"), "/tmp"):
            if os.path.isdir(cand) and _free_bytes(cand) >= need:
                d = cand
                break
        if d is None:
            raise RuntimeError("no filesystem for the shared .lfm: need %.2f GB free in /dev/shm or /tmp" % (need / 1e9))
        self.path = os.path.join(d, "lfm_bench_%s_%d_%d.lfm" % (port, world, os.getuid()))
        self.rank = rank
        if rank == 0:
            with open(self.path, "wb") as f:
                f.truncate(cap)
        dist.barrier()
        self.buf = np.memmap(self.path, dtype=np.uint8, mode="r+", shape=(cap,))
        self.len = 0

    def close(self):
        del self.buf
        if self.rank == 0:
            try:
                os.unlink(self.path)
            except OSError:
                pass


def place_in_shared(shm, b, rank, world, total_z, backend, threads):
    """all_gather of (payload bytes, blocks) per slab, then this rank's blocks
    and offset-table entries into the shared .lfm (lfm.place_slab)."""
    pb, nb = lfm.slab_info(b)
    dev = "cuda" if backend == "nccl" else "cpu"
    mine = torch.tensor([pb, nb], dtype=torch.int64, device=dev)
    every = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(every, mine)
    sizes = torch.stack(every).cpu().tolist()
    payload_off = sum(x[0] for x in sizes[:rank])
    block_idx = sum(x[1] for x in sizes[:rank])
    total_blocks = sum(x[1] for x in sizes)
    lfm.place_slab(b, shm.buf, total_z, total_blocks, block_idx, payload_off, threads)
    shm.len = 320 + 8 * total_blocks + sum(x[0] for x in sizes)


def host_input_rates(enc, d_img, zf, steps=2, psteps=6):
    """PCIe-inclusive encode: the stack in host memory (pinned, then pageable),
    uploaded by the encoder inside the timed region (selection included):
    one synchronous encode at a time (lfm_encoder_encode, what writeKLBstack
    does per call), and pipelined submit / wait (a caller streaming stacks:
    each stack's upload runs under the previous stack's GPU bzip2); the last
    pipelined .lfm is compared with the synchronous one."""
    out = {}
    h_pin = torch.empty(tuple(d_img.shape), dtype=torch.int16, pin_memory=True)
    h_pin.copy_(d_img)
    arrays = (("pinned", h_pin.numpy().view(np.uint16)), ("pageable", np.array(h_pin.numpy().view(np.uint16))))
    for name, arr in arrays:
        ref = bytes(enc.encode(arr, header_version=0, nnum=T, copy=False)[0])  # warm
        t0 = time.perf_counter()
        h2d = 0.0
        for _ in range(steps):
            _, st = enc.encode(arr, header_version=0, nnum=T, copy=False)
            h2d += st["h2d_ms"]
        dt = (time.perf_counter() - t0) / steps
        res = {"Mpixel_per_s": round(X * Y * zf / dt / 1e6, 1), "ms_per_step": round(dt * 1e3, 2),
               "h2d_ms": round(h2d / steps, 2)}
        # pipelined: two stacks in flight
        pending = enc.submit(arr, header_version=0, nnum=T)
        enc.wait(pending, copy=False)
        t0 = time.perf_counter()
        pending = None
        for _ in range(psteps):
            t = enc.submit(arr, header_version=0, nnum=T)
            if pending is not None:
                enc.wait(pending, copy=False)
            pending = t
        b, _ = enc.wait(pending, copy=False)
        dtp = (time.perf_counter() - t0) / psteps
        same = bytes(b) == ref  # the last pipelined .lfm (outside the timed region)
        res["pipelined"] = {"Mpixel_per_s": round(X * Y * zf / dtp / 1e6, 1), "ms_per_step": round(dtp * 1e3, 2),
                            "same_bytes": same}
        out[name] = res
    out["note"] = ("host stack -> in-memory .lfm, H2D inside the timed region (chunked upload overlapped with the "
                   "predictor and GPU bzip2); value above is HBM-resident")
    return out


def config5_leg(local, threads, nvol=4):
    """Config 5 at full frame size on this GPU: nvol t-volumes of the 4096 x
    4096 x 32 video stack (tiles, Nnum 13, auto-selected on volume 0's frame
    0), resident in HBM, encoded into ONE .lfm (predictor per volume + GPU
    bzip2 + D2H), SHA-256 checked against the oracle (cfg5x4); then decoded
    (GPU bzip2 decode + GPU inverse predictor + D2H into a fresh host array)
    and compared with the input.  SURVEY 8(d) config 5 is the 100-volume
    encode + decode round trip; every volume codes alone, so this is its
    per-GPU rate."""
    X5, Y5, Z5, T5, seed = 4096, 4096, 32, 13, 0x4C464D05
    e = _manifest("cfg5x4_4096x4096x32x1x4_video_tiles_auto")
    d = torch.empty((nvol, 1, Z5, Y5, X5), dtype=torch.int16, device="cuda")
    for t in range(nvol):
        lfm.synth_device(d[t, 0], X5, Y5, Z5, T5, t_index=t, idx0=t * Z5 * X5 * Y5, seed=seed)
    torch.cuda.synchronize()
    lfm.set_family("tiles")
    px = nvol * X5 * Y5 * Z5
    enc = lfm.Encoder(device=local, num_threads=threads)
    try:
        enc.encode(d, header_version=0x80, nnum=T5, copy=False)  # warm: buffers sized and first-touched
        runs = []
        for _ in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            b, st = enc.encode(d, header_version=0x80, nnum=T5, copy=False)
            runs.append((time.perf_counter() - t0) * 1e3)
        buf = bytes(b)
    finally:
        enc.close()
    ok = None
    if e is not None and nvol == e["xyzct"][4]:
        ok = hashlib.sha256(buf).hexdigest() == e["sha256"] and len(buf) == e["size"]
    ref = d.cpu().numpy().view(np.uint16)
    del d
    dl = []
    exact = True
    for _ in range(2):
        t0 = time.perf_counter()
        img = lfm.decode(buf, num_threads=threads)
        dl.append((time.perf_counter() - t0) * 1e3)
        exact = exact and bool(np.array_equal(img.reshape(ref.shape), ref))
        del img
    lfm.set_family(FAMILY)
    ems, dms = min(runs), dl[-1]
    return {"workload": "%d t-volumes of config 5 (4096x4096x32x1x%d, video bit, tiles, Nnum 13, auto), one .lfm"
                        % (nvol, nvol),
            "encode_Mpixel_per_s": round(px / ems / 1e3, 1), "encode_ms": round(ems, 2),
            "encode_runs_ms": [round(x, 2) for x in runs], "chosen_predictor": st["chosen"],
            "ratio": round(px * 2 / len(buf), 4),
            "verified": {"against": "cfg5x4 whole-file SHA-256 (oracle, reference bzip2-1.0.6)", "ok": ok},
            "decode_Mpixel_per_s": round(px / dms / 1e3, 1), "decode_ms": round(dms, 1),
            "decode_runs_ms": [round(x, 1) for x in dl], "decode_exact": exact,
            "round_trip_Mpixel_per_s": round(px / (ems + dms) / 1e3, 1),
            "note": "encode from HBM to the in-memory .lfm; decode from the in-memory .lfm to a host array (PCIe "
                    "upload of the payload and download of the pixels included)"}


def config5_host_leg(local, threads, nvol):
    """Config 5 streamed from HOST memory through the drop-in writer and
    reader: nvol t-volumes of the 4096 x 4096 x 32 video stack (tiles, Nnum
    13, auto) in one host array -> lfm_encoder_encode_multi (the block
    scheduler behind klb_imageIO::writeImage; t-volumes farmed over the
    visible devices, chunked uploads overlapped with the predictor and GPU
    bzip2) -> one in-memory .lfm; volumes 0..3 and, when present, 50 and 99
    SHA-256-checked against the oracle (cfg5x4, cfg5far: the far ones lie
    past 2^32 in the offset table), then the host input is released and every volume is
    read back on its own (lfm_decode_memory_roi, readKLBroiInPlace's path)
    and compared with its regenerated pixels.  Peak RSS is the process's."""
    import resource
    X5, Y5, Z5, T5, seed = 4096, 4096, 32, 13, 0x4C464D05
    e = _manifest("cfg5x4_4096x4096x32x1x4_video_tiles_auto")
    img = np.empty((nvol, 1, Z5, Y5, X5), dtype=np.uint16)
    d = torch.empty((Z5, Y5, X5), dtype=torch.int16, device="cuda")
    for t in range(nvol):
        lfm.synth_device(d, X5, Y5, Z5, T5, t_index=t, idx0=t * Z5 * X5 * Y5, seed=seed)
        torch.from_numpy(img[t, 0].view(np.int16)).copy_(d)
        if t % 10 == 9:
            print("config5_host: %d / %d volumes generated" % (t + 1, nvol), file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    lfm.set_family("tiles")
    px = nvol * X5 * Y5 * Z5
    enc = lfm.Encoder(device=local, num_threads=threads)
    out = {"workload": "%d t-volumes of config 5 (4096x4096x32x1x%d, video, tiles, Nnum 13, auto) from host memory"
                       % (nvol, nvol),
           "path": "lfm_encoder_encode_multi (klb_imageIO::writeImage's scheduler, devices %s) -> in-memory .lfm; "
                   "per-volume lfm_decode_memory_roi" % lfm.get_devices()}
    try:
        # one untimed volume first: device buffers, pinned staging and the
        # writer's threads are set up once per process, as in a long acquisition
        enc.encode_multi(img[:1], header_version=0x80, nnum=T5, copy=True)
        # two timed calls: the first also allocates and first-touches the
        # device buffers for the whole stack; the second is the steady state
        # of a writer that is called again with stacks of the same shape
        enc_runs = []
        for _ in range(2):
            t0 = time.perf_counter()
            b, st = enc.encode_multi(img, header_version=0x80, nnum=T5, copy=False)
            enc_runs.append(time.perf_counter() - t0)
            print("config5_host: encoded in %.2f s" % enc_runs[-1], file=sys.stderr, flush=True)
        enc_s = enc_runs[-1]
        nb = 4 * 43 * 43  # blocks per volume (96 x 96 x 8)
        offs = np.frombuffer(b, dtype="<u8", count=nvol * nb, offset=320)
        base, prev, sha_ok = 320 + 8 * nvol * nb, 0, None
        checked = []
        if e is not None:
            sha_ok = True
            for t in range(min(4, nvol)):
                end = int(offs[(t + 1) * nb - 1])
                sha_ok = sha_ok and hashlib.sha256(b[base + prev:base + end]).hexdigest() == e["volume_sha256"][t]
                checked.append(t)
                prev = end
        # far volumes (t = 50, 99 of the 100-volume stack): streams at u64
        # end-offsets past 2^32 against the oracle's per-volume digests
        far = _manifest("cfg5far_4096x4096x32x1x100_video_tiles_auto")
        far_max_offset = 0
        if far is not None:
            for ts, want in far["volumes"].items():
                t = int(ts)
                if t >= nvol:
                    continue
                a0 = int(offs[t * nb - 1]) if t else 0
                a1 = int(offs[(t + 1) * nb - 1])
                got = hashlib.sha256(b[base + a0:base + a1]).hexdigest() == want["sha256"] and a1 - a0 == want["bytes"]
                sha_ok = (sha_ok is not False) and got
                checked.append(t)
                far_max_offset = max(far_max_offset, a1)
        lfm_bytes = len(b)
        del img
        exact, dec_s = True, 0.0
        vbuf = np.empty((Z5, Y5, X5), dtype=np.uint16)  # the reader's own buffer, reused per volume
        vbuf.fill(0)
        for t in range(nvol):
            t1 = time.perf_counter()
            v = lfm.decode_roi(b, [0, 0, 0, 0, t], [X5 - 1, Y5 - 1, Z5 - 1, 0, t], num_threads=threads, out=vbuf)
            dec_s += time.perf_counter() - t1
            lfm.synth_device(d, X5, Y5, Z5, T5, t_index=t, idx0=t * Z5 * X5 * Y5, seed=seed)
            exact = exact and bool(np.array_equal(v.reshape(Z5, Y5, X5), d.cpu().numpy().view(np.uint16)))
            del v
            if t % 10 == 9:
                print("config5_host: %d / %d volumes read back" % (t + 1, nvol), file=sys.stderr, flush=True)
    finally:
        enc.close()
        lfm.release_encoders()
        lfm.set_family(FAMILY)
    out.update({"volumes": nvol, "encode_Mpixel_per_s": round(px / enc_s / 1e6, 1), "encode_s": round(enc_s, 3),
                "encode_first_call_s": round(enc_runs[0], 3),
                "h2d_ms": round(st["h2d_ms"], 1), "ratio": round(px * 2 / lfm_bytes, 4),
                "verified": {"against": "per-volume SHA-256 of volumes %s (cfg5x4 / cfg5far manifests: oracle, "
                                        "reference bzip2-1.0.6)" % checked, "ok": sha_ok,
                             "max_checked_end_offset": far_max_offset},
                "decode_Mpixel_per_s": round(px / dec_s / 1e6, 1), "decode_s": round(dec_s, 3),
                "decode_exact": exact,
                "peak_rss_GB": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024 / 1e9, 2),
                "input_GB": round(px * 2 / 1e9, 2), "lfm_GB": round(lfm_bytes / 1e9, 2)})
    return out


def _lfm_manifest(name):
    path = os.path.join(REPO, "tests", "golden", "lfm_manifest.json")
    try:
        return {e["name"]: e for e in json.load(open(path))}.get(name)
    except (OSError, ValueError):
        return None


def small_configs_leg(local, threads, reps=20):
    """BASELINE.md's per-config figures for the two small configs.
    Config 1 (testData/img.tif page 0, 101 x 151, all zeros; and its 29-page
    stack; request 8 = predictor off): this library's encode of the host
    image, Mpixel/s and ratio, bytes checked (the reference's CPU path on the
    same input is timed in cpu_baseline).
    Config 2 (512 x 512, Nnum 13, space, auto): device-resident encode and the
    predictor kernel's HBM fraction (a 0.5 MB frame: launch-latency bound)."""
    out = {}
    tif = np.load(os.path.join(REPO, "tests", "golden", "img_tif.npz"))["img"]
    enc = lfm.Encoder(device=local, num_threads=threads)
    try:
        lfm.set_family("tiles")
        for name, img in (("cfg1_imgtif_page0_req8", tif[0][None, None, None]),
                          ("cfg1_imgtif_stack_req8", tif[None, None])):
            e = _lfm_manifest(name)
            px = int(np.prod(img.shape))
            b, _ = enc.encode(img, header_version=8, nnum=13)
            t0 = time.perf_counter()
            for _ in range(reps):
                b, _ = enc.encode(img, header_version=8, nnum=13)
            ms = (time.perf_counter() - t0) * 1e3 / reps
            ok = None if e is None else hashlib.sha256(b).hexdigest() == e["sha256"]
            out[name] = {"shape_tczyx": list(img.shape), "Mpixel_per_s": round(px / ms / 1e3, 2),
                         "ms": round(ms, 3), "ratio": round(px * 2 / len(b), 4), "verified": ok,
                         "note": "host image -> in-memory .lfm (the reference's CPU path on the same input: "
                                 "cpu_baseline.config1)"}
        lfm.set_family("space")
        e = _lfm_manifest("cfg2_512x512_space_auto")
        d = torch.empty((1, 512, 512), dtype=torch.int16, device="cuda")
        lfm.synth_device(d, 512, 512, 1, 13, seed=0x4C464D02)
        torch.cuda.synchronize()
        b, st = enc.encode(d, header_version=0, nnum=13)
        pms, walls = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            b, st = enc.encode(d, header_version=0, nnum=13)
            walls.append((time.perf_counter() - t0) * 1e3)
            pms.append(st["predict_ms"])
        ms, kms = float(np.median(walls)), float(np.median(pms))
        alg = 512 * 512 * 4
        out["cfg2_512x512_space_auto"] = {
            "Mpixel_per_s": round(512 * 512 / ms / 1e3, 2), "ms": round(ms, 3), "chosen_predictor": st["chosen"],
            "ratio": round(512 * 512 * 2 / len(b), 4),
            "verified": None if e is None else hashlib.sha256(b).hexdigest() == e["sha256"],
            "predict_kernel_ms": round(kms, 4), "predict_frac_8TBs": round(alg / (kms / 1e3) / 8e12, 4),
            "note": "one 512x512 frame: the encode is latency-bound (selection, one predictor launch, one bzip2 "
                    "batch); the kernel moves 1 MiB, far below what fills the GPU"}
    finally:
        enc.close()
        lfm.set_family(FAMILY)
    return out


def inproc_leg(local, threads, ndevs):
    """The drop-in multi-GPU writer -- lfm_encoder_encode_multi, the block
    scheduler behind klb_imageIO::writeImage / writeKLBstack -- on config 4
    (2048 x 2048 x 256 uint16, tiles, Nnum 15, auto) from HOST memory: z-slabs
    of whole block layers farmed to each device list in ndevs, one host thread
    per device, in-order writer; PCIe-inclusive; SHA-256 checked (cfg4)."""
    X4, Y4, Z4, T4, seed = 2048, 2048, 256, 15, 0x4C464D04
    e = _manifest("cfg4_2048x2048x256_tiles_auto")
    d = torch.empty((Z4, Y4, X4), dtype=torch.int16, device="cuda")
    lfm.synth_device(d, X4, Y4, Z4, T4, seed=seed)
    host = torch.empty((Z4, Y4, X4), dtype=torch.int16, pin_memory=True)
    host.copy_(d)
    del d
    arr = host.numpy().view(np.uint16)
    lfm.set_family("tiles")
    out = {"workload": "config 4: 2048x2048x256 uint16 from host memory, tiles, Nnum 15, auto, 96x96x8 blocks",
           "path": "lfm_encoder_encode_multi (klb_imageIO::writeImage's scheduler): z-slabs per device, in-order "
                   "writer, H2D inside the timed region"}
    px = X4 * Y4 * Z4
    enc = lfm.Encoder(device=local, num_threads=threads)
    try:
        for devs in ndevs:
            lfm.set_devices(devs)
            b, _ = enc.encode_multi(arr, header_version=0, nnum=T4, copy=False)  # warm (per-device encoders)
            runs = []
            for _ in range(2):
                t0 = time.perf_counter()
                b, st = enc.encode_multi(arr, header_version=0, nnum=T4, copy=False)
                runs.append((time.perf_counter() - t0) * 1e3)
            ok = None if e is None else (len(b) == e["size"] and hashlib.sha256(b).hexdigest() == e["sha256"])
            ms = min(runs)
            out["workers_%d" % len(devs) if len(set(devs)) < len(devs) else "gpus_%d" % len(devs)] = {"devices": devs, "Mpixel_per_s": round(px / ms / 1e3, 1),
                                          "ms": round(ms, 2), "runs_ms": [round(x, 2) for x in runs],
                                          "verified": ok}
    finally:
        lfm.set_devices([])
        enc.close()
        lfm.release_encoders()
        lfm.set_family(FAMILY)
    return out


def torchrun_cmd(n, argv, port):
    """The child command `bench.py --gpus N` runs when it is not already one
    rank of an N-rank job: torchrun with N ranks on this node (127.0.0.1
    rendezvous), bench.py with the same arguments."""
    return [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % n,
            "--master-addr=127.0.0.1", "--master-port=%d" % port, os.path.abspath(__file__)] + list(argv)


def launch_ranks(n, argv):
    """Start the N rank processes as children (torchrun) and exit with their
    status.  Called before anything touches the GPU: this process only counts
    devices (no HIP context) and never execs; rank 0's JSON line reaches the
    caller through the inherited stdout."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    sys.stdout.flush()
    return subprocess.run(torchrun_cmd(n, argv, port), env=env).returncode


def rank_layout(gpus, env, ndev):
    """(world, rank, local, local_world) of this process, or an error string.
    --gpus N is authoritative: a process with no WORLD_SIZE and N > 1 launches
    N ranks (returned as world None), and a rank whose WORLD_SIZE differs from
    N refuses to run (its line would be labelled with the wrong GPU count)."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        if gpus > 1:
            backend = env.get("LFM_BENCH_BACKEND", "nccl")
            if backend == "nccl" and gpus > ndev:
                return "--gpus %d but only %d device(s) visible" % (gpus, ndev)
            return None, 0, 0, gpus
        if gpus < 1:
            return "--gpus must be >= 1"
        return 1, 0, 0, 1
    world = int(ws)
    if world != gpus:
        return "WORLD_SIZE=%d but --gpus %d: the line would misreport the GPU count" % (world, gpus)
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", "0"))
    return world, rank, local, int(env.get("LOCAL_WORLD_SIZE", str(world)))


def predictor_standalone(d_img, zf, k, alg_bytes, launches=20):
    """The roofline kernel with the GPU to itself: `launches` launches of the
    config-3 predictor over the resident stack on one HIP stream, timed one by
    one with HIP events on that stream.  "warm": back to back; "flushed": a
    1 GiB device fill before each launch (on the same stream, outside its
    events), so each launch starts with the caches holding someone else's
    dirty lines, as in the encode.  "copies": the same two protocols for plain
    copies of the same bytes (the stack read once, as many bytes written) on
    the same box -- the ceiling a streaming kernel of this traffic reaches
    here: hipMemcpyAsync device to device and torch's elementwise add."""
    sym = torch.empty_like(d_img)
    scratch = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    st = torch.cuda.Stream()
    out = {"launches": launches, "predictor": k, "algorithmic_bytes": alg_bytes}

    def timed(fn):
        res = {}
        for mode in ("warm", "flushed"):
            ms = []
            for i in range(launches + 2):
                if mode == "flushed":
                    scratch.fill_(i & 0xFF)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                fn()
                e1.record(st)
                e1.synchronize()
                if i >= 2:
                    ms.append(e0.elapsed_time(e1))
            med = float(np.median(ms))
            res[mode] = {"kernel_ms_median": round(med, 4), "kernel_ms_min": round(float(min(ms)), 4),
                         "frac": round(alg_bytes / (med / 1e3) / 1e9 / PEAK_HBM_GBS, 4)}
        return res

    with torch.cuda.stream(st):
        out.update(timed(lambda: lfm.predict_device(d_img, sym, X, Y, zf, T, FAMILY, k, stream=st)))
        out["copies"] = {"hipMemcpy_d2d": timed(lambda: sym.copy_(d_img)),
                         "torch_add": timed(lambda: torch.add(d_img, 1, out=sym))}
    st.synchronize()
    for mode in ("warm", "flushed"):
        best = max(c[mode]["frac"] for c in out["copies"].values())
        out[mode]["vs_best_copy"] = round(out[mode]["frac"] / best, 4) if best > 0 else None
    del scratch, sym
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--frames", type=int, default=Z)
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--no-host-input", action="store_true")
    ap.add_argument("--no-config5", action="store_true")
    ap.add_argument("--no-small", action="store_true")
    ap.add_argument("--no-inproc", action="store_true")
    ap.add_argument("--config5-host-volumes", type=int, default=8,
                    help="t-volumes of the config5_host leg (N = 1; 0: skip); the full stack is 100")
    ap.add_argument("--only-config5-host", action="store_true",
                    help="skip the timed encode and every other leg (a long config5_host run)")
    args = ap.parse_args()

    # device_count() creates no HIP context on this image: safe before the spawn
    lay = rank_layout(args.gpus, os.environ, torch.cuda.device_count())
    if isinstance(lay, str):
        print("bench.py: " + lay, file=sys.stderr)
        sys.exit(2)
    world, rank, local, local_world = lay
    if world is None:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    # LFM_BENCH_BACKEND=gloo rehearses the N-rank path with several ranks on
    # one GPU (local rank modulo the visible devices); the driver's N-GPU runs
    # use nccl (RCCL): the barriers, the slab-size all_gather and the MAX
    backend = os.environ.get("LFM_BENCH_BACKEND", "nccl")
    ndev = max(1, torch.cuda.device_count())
    local = local % ndev
    torch.cuda.set_device(local)
    cpu_group = None
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            # host-side waits while rank 0 drives every device (the inproc leg):
            # an RCCL barrier would park a spinning kernel on each waiting GPU
            cpu_group = dist.new_group(backend="gloo")
        else:
            dist.init_process_group(backend)
            cpu_group = dist.group.WORLD
    lfm.require_gpu()
    lfm.set_family(FAMILY)
    zf = args.frames
    threads = host_threads(local_world)
    if args.only_config5_host:
        if world > 1 or args.config5_host_volumes < 1:
            print("bench.py: --only-config5-host runs one process with --config5-host-volumes >= 1", file=sys.stderr)
            sys.exit(2)
        print(json.dumps({"config5_host": config5_host_leg(local, threads, args.config5_host_volumes)}), flush=True)
        return

    d_img = torch.empty((zf, Y, X), dtype=torch.int16, device="cuda")
    # rank r holds z-slab r (frames r*zf .. r*zf+zf-1) of a (world * zf)-frame stack
    z0 = rank * zf
    lfm.synth_device(d_img, X, Y, zf, T, z0=z0, seed=SEED)
    if rank == 0:
        sel_frame = None  # frame 0 of the slab is the stack's
    else:  # the stack's frame 0, for the redundant selection
        sel_frame = torch.empty((1, Y, X), dtype=torch.int16, device="cuda")
        lfm.synth_device(sel_frame, X, Y, 1, T, z0=0, seed=SEED)
    torch.cuda.synchronize()
    enc = lfm.Encoder(device=local, num_threads=threads)
    shm = None
    if world > 1:
        nb_total = world * ((X + 95) // 96) * ((Y + 95) // 96) * ((zf + 7) // 8)
        shm = SharedLfm(rank, world, 320 + 8 * nb_total + world * (X * Y * zf * 2 * 103 // 100 + (1 << 20)))

    place_ms = []

    def finish(ticket, stats):
        # the .lfm stays in the encoder's buffer (no copy into a Python bytes object)
        b, st = enc.wait(ticket, copy=False)
        if shm is not None:
            t1 = time.perf_counter()
            place_in_shared(shm, b, rank, world, world * zf, backend, threads)
            place_ms.append((time.perf_counter() - t1) * 1e3)
        stats.append(st)
        return b

    # LFM_BENCH_FORCE_K=k (diagnostic, not the metric): skip the selection and
    # force predictor k, to see what the selection costs the pipeline
    hv_req = 8 + int(os.environ["LFM_BENCH_FORCE_K"]) if os.environ.get("LFM_BENCH_FORCE_K") else 0

    def run(nsteps, stats):
        """nsteps encodes of the stack, pipelined (lfm_encoder_submit / wait):
        encode i's kernels run while encode i-1's last payload copies drain
        over PCIe; every .lfm is complete when its wait returns."""
        pending = None
        b = None
        for _ in range(nsteps):
            # auto request: the submit selects on the stack's frame 0 (its own
            # frame 0 at rank 0, handed in on the others) on the encoder's
            # stream, after the previous encode's kernels
            ticket = enc.submit(d_img, z0, header_version=hv_req, nnum=T, select_frame=sel_frame)
            if pending is not None:
                b = finish(pending, stats)
            pending = ticket
        return finish(pending, stats) if pending is not None else None

    run(args.warmup, [])
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    b = run(args.steps, stats)
    out_len = b.nbytes
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    # one unpipelined encode (select + encode + every copy, nothing in flight), for its latency
    t1 = time.perf_counter()
    _, lat_st = enc.wait(enc.submit(d_img, z0, header_version=0, nnum=T, select_frame=sel_frame), copy=False)
    latency_ms = max_over_ranks(time.perf_counter() - t1) * 1e3

    px_rank = X * Y * zf
    value = world * px_rank * args.steps / elapsed / 1e6
    pred_ms = float(np.mean([s["predict_ms"] for s in stats]))
    alg_bytes = px_rank * 4  # 2 B read + 2 B written per pixel (no temporal frames in this config)
    achieved = alg_bytes / (pred_ms / 1e3) / 1e9
    traffic = None
    # the newest PMC traffic file of the kernel (rocprofv3 --pmc FETCH_SIZE /
    # WRITE_SIZE passes over scripts/encode_probe.py, scripts/pmc_summary.py)
    tpath = None
    for name in ("r06_traffic_predict.json", "r05_traffic_predict.json", "r04_traffic_predict.json", "r03_traffic_predict.json"):
        tpath = os.path.join(REPO, "profiles", name)
        if os.path.exists(tpath):
            break
    if os.path.exists(tpath):
        try:
            traffic = json.load(open(tpath)).get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    line = {
        "metric": "uint16 Mpixel/s encode (predictor->bzip2) at 1/2/4/8 GPUs; ratio parity",
        "value": round(value, 3),
        "unit": "Mpixel/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic (SURVEY 8(d) integer light-field generator, generated on device)",
        "config": {"workload": "config 3: %dx%dx%d uint16 stack per GPU, Nnum %d, %s family, predictor auto-selected "
                               "on frame 0, 96x96x8 blocks, bzip2, in-memory .lfm%s" % (
                                   X, Y, zf, T, FAMILY,
                                   "" if world == 1 else " of the whole %d-frame stack in host shared memory"
                                   % (world * zf)),
                   "parallelism": "z-slab per GPU (slab-size all_gather only)", "host_threads_per_gpu": threads},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                     "kernel": "lfm::predict_vec<1,K,15,1,4,1,3> (fused angle predictor + symbolize, 8 pixels "
                               "per lane, %d frames per launch)" % zf,
                     "traffic_file": os.path.relpath(tpath, REPO) if traffic is not None else None,
                     "kernel_ms": round(pred_ms, 4), "algorithmic_bytes": alg_bytes,
                     "read_only_frac": round(px_rank * 2 / (pred_ms / 1e3) / 1e9 / PEAK_HBM_GBS, 4),
                     # the timed region's launches share the CUs with the previous
                     # encode's bzip2 tail (the next predictor stage starts before
                     # that encode is released); the unpipelined latency encode's
                     # launch has the GPU to itself
                     "kernel_ms_alone": round(float(lat_st["predict_ms"]), 4),
                     "frac_alone": round(alg_bytes / (float(lat_st["predict_ms"]) / 1e3) / 1e9 / PEAK_HBM_GBS, 4)},
        "stages_ms": {k: round(float(np.mean([s[k] for s in stats])), 3)
                      for k in ("select_ms", "predict_ms", "d2h_ms", "compress_ms", "total_ms")},
        "pipelined": "two encodes in flight (lfm_encoder_submit / wait): an encode's kernels overlap the previous "
                     ".lfm's last payload copies; every .lfm is complete inside the timed region",
        "latency_ms_per_encode": round(latency_ms, 3),
        "chosen_predictor": stats[-1]["chosen"],
        "ratio": round(px_rank * 2 / out_len, 4),
    }
    if place_ms:
        line["stages_ms"]["place_ms"] = round(float(np.mean(place_ms[-args.steps:])), 3)
    # GPU bzip2 stages (HIP events per HIP stream, max over the two streams that
    # run concurrently) and their rate in block bytes
    bz_in = stats[-1]["bz_in_bytes"]
    for name in ("rle1", "bwt", "mtf", "huffman", "emit"):
        ms = float(np.mean([s["bz_stage_ms"][name] for s in stats]))
        line["stages_ms"]["bz_%s_ms" % name] = round(ms, 3)
        line["stages_ms"]["bz_%s_GBps" % name] = round(bz_in / (ms / 1e3) / 1e9, 1) if ms > 0 else None
    # byte check of the last timed .lfm against the oracle (outside the timed region)
    if rank == 0:
        buf = b if shm is None else shm.buf[:shm.len]
        line["verified"] = verify_lfm(buf, world, zf)
        if world > 1:
            line["ratio"] = round(world * px_rank * 2 / shm.len, 4)
    if world > 1:
        dist.barrier()
        shm.close()
        if not args.no_inproc:
            # the drop-in writer over all N devices, driven from rank 0 alone
            # (what a writeKLBstack / MEX caller on this node gets): every rank
            # first releases its encoder and device memory
            enc.close()
            del d_img
            sel_frame = None
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
            dist.barrier(group=cpu_group)
            if rank == 0:
                devs = [r % ndev for r in range(world)]
                node_threads = min(len(os.sched_getaffinity(0)), threads * local_world)
                line["inproc"] = inproc_leg(local, node_threads if backend == "nccl" else threads,
                                            [[local], devs])
            dist.barrier(group=cpu_group)
    if rank == 0 and world == 1:
        line["roofline"]["standalone"] = predictor_standalone(d_img, zf, int(stats[-1]["chosen"]) & 0x7F, alg_bytes)
    buf = bytes(b) if rank == 0 and world == 1 and not args.no_decode else None  # before b's buffer is reused
    if rank == 0 and world == 1 and not args.no_host_input:
        line["host_input"] = host_input_rates(enc, d_img, zf)
    if buf is not None:
        # the decode is a reader's job: it runs after the encoder (its buffers,
        # pinned output and finisher threads) is released, as in a separate
        # reader process
        enc.close()
        ref = d_img.cpu().numpy().view(np.uint16)
        # five decodes, each into a fresh array (its first-touch page faults
        # timed): the first also pays one-time costs (lazily loaded kernels,
        # the decoder's device buffers and pinned staging) and the GPU page-
        # table updates of the frees and the pageable copy just above, which
        # hold up its first DMA; "ms" is the median
        dlist, exact = [], True
        for _ in range(5):
            t1 = time.perf_counter()
            img = lfm.decode(buf, num_threads=threads)
            dlist.append((time.perf_counter() - t1) * 1e3)
            exact = exact and bool(np.array_equal(img.reshape(ref.shape), ref))
            del img
        dms = float(np.median(dlist))
        line["decode"] = {"ms": round(dms, 1), "Mpixel_per_s": round(px_rank / dms / 1e3, 1),
                          "first_ms": round(dlist[0], 1), "runs_ms": [round(x, 1) for x in dlist],
                          "exact": exact,
                          "path": "GPU bzip2 decode + GPU inverse predictor (host libbz2 only for flagged streams, %d threads)" % threads}
    if rank == 0 and world == 1 and not args.no_small:
        line["configs_1_2"] = small_configs_leg(local, threads)
    if rank == 0 and world == 1 and not args.no_config5:
        line["config5"] = config5_leg(local, threads)
    if rank == 0 and world == 1 and args.config5_host_volumes > 0:
        line["config5_host"] = config5_host_leg(local, threads, args.config5_host_volumes)
    if rank == 0 and world == 1 and not args.no_inproc:
        nvis = torch.cuda.device_count()
        legs = [[local]] + ([list(range(nvis))] if nvis > 1 else [])
        if os.environ.get("LFM_BENCH_INPROC"):  # e.g. "0,0,0,0": four workers on one GPU (rehearsal)
            legs = [[local], [int(x) for x in os.environ["LFM_BENCH_INPROC"].split(",")]]
        line["inproc"] = inproc_leg(local, threads, legs)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(threads=threads)
        line["cpu_baseline"]["affinity_cpus"] = len(os.sched_getaffinity(0))
        line["cpu_baseline"]["threads_note"] = (
            "cores = the threads used: this process's CPU share, min(affinity, OMP_NUM_THREADS=%s); "
            "the box's affinity mask shows every host CPU, the job's share is OMP_NUM_THREADS"
            % os.environ.get("OMP_NUM_THREADS", "unset"))
    if rank == 0:
        print(json.dumps(line), flush=True)
    enc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
