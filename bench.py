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

Multi-GPU (torchrun, one process per GPU): rank r encodes z-slab r of a
(world x 64)-frame stack (lfm.shard: slabs are whole blocks deep, so the slab
files join byte-identically with lfm.merge_slabs, tests/test_shard_cpu.py);
the predictor is selected on the stack's frame 0 redundantly on every rank
(no broadcast) and forced for the slab; no data-path collective (scaling
"weak"); a barrier + MAX-over-ranks of the timed region gives value.

Also reported: `roofline` of the dominant kernel (fused predictor, HIP-event
time per launch on its own stream) and `cpu_baseline` = the reference's CPU
bzip2-only path (request 8, same blocks, the reference's own bzip2-1.0.6 from
oracle/_ref) on a bounded sample, timed on this host.
"""
import argparse
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
from lfm.shard import forced_request, max_over_ranks  # noqa: E402

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
    return {"value": px / dt / 1e6, "unit": "Mpixel/s", "cores": threads,
            "kind": "reference" if "reference" in bz.kind else "port",
            "sample": "%dx%dx%d uint16 synthetic slab of the bench stack, request 8 (predictor off), 96x96x8 blocks, "
                      "bzip2 level 2 (%s), %d blocks, ratio %.3f" % (X, Y, zs, bz.kind, len(blocks),
                                                                      px * 2 / total),
            "value_1thread": px1 / dt1 / 1e6, "nproc": os.cpu_count()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--frames", type=int, default=Z)
    ap.add_argument("--no-decode", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    # LFM_BENCH_BACKEND=gloo rehearses the N-rank path with several ranks on
    # one GPU (local rank modulo the visible devices); the driver's N-GPU runs
    # use nccl (RCCL), which only carries the barriers and the MAX reduction
    backend = os.environ.get("LFM_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    lfm.require_gpu()
    lfm.set_family(FAMILY)
    zf = args.frames
    threads = host_threads(local_world)

    d_img = torch.empty((zf, Y, X), dtype=torch.int16, device="cuda")
    # rank r holds z-slab r of a (world * zf)-frame stack
    z0 = rank * zf
    lfm.synth_device(d_img, X, Y, zf, T, t_index=0, idx0=z0 * X * Y, seed=SEED)
    if rank == 0:
        d_f0 = d_img[0]
    else:  # the stack's frame 0, for the redundant selection
        d_f0 = torch.empty((1, Y, X), dtype=torch.int16, device="cuda")
        lfm.synth_device(d_f0, X, Y, 1, T, t_index=0, idx0=0, seed=SEED)
    torch.cuda.synchronize()
    enc = lfm.Encoder(device=local, num_threads=threads)

    def step():
        t0 = time.perf_counter()
        k, _ = lfm.select_device(d_f0, X, Y, T, FAMILY)  # selection on the stack's frame 0
        sel_ms = (time.perf_counter() - t0) * 1e3
        # the .lfm stays in the encoder's buffer (no copy into a Python bytes object)
        b, st = enc.encode_slab(d_img, z0, header_version=forced_request(k), nnum=T, copy=False)
        st["select_ms"] = sel_ms
        st["total_ms"] += sel_ms
        return b, st

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    stats = []
    out_len = 0
    for _ in range(args.steps):
        b, st = step()
        stats.append(st)
        out_len = b.nbytes
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)

    px_rank = X * Y * zf
    value = world * px_rank * args.steps / elapsed / 1e6
    pred_ms = float(np.mean([s["predict_ms"] for s in stats]))
    alg_bytes = px_rank * 4  # 2 B read + 2 B written per pixel (no temporal frames in this config)
    achieved = alg_bytes / (pred_ms / 1e3) / 1e9
    traffic = None
    tpath = os.path.join(REPO, "profiles", "r01_traffic_predict.json")
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
                               "on frame 0, 96x96x8 blocks, bzip2, in-memory .lfm" % (X, Y, zf, T, FAMILY),
                   "parallelism": "z-slab per GPU (no collective)", "host_threads_per_gpu": threads},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBS, 4), "traffic": traffic,
                     "kernel": "lfm::predict_ring<1,K,4,1,3> (fused angle predictor + symbolize, %d frames per "
                               "launch)" % zf,
                     "kernel_ms": round(pred_ms, 4), "algorithmic_bytes": alg_bytes,
                     "read_only_frac": round(px_rank * 2 / (pred_ms / 1e3) / 1e9 / PEAK_HBM_GBS, 4)},
        "stages_ms": {k: round(float(np.mean([s[k] for s in stats])), 3)
                      for k in ("select_ms", "predict_ms", "d2h_ms", "compress_ms", "total_ms")},
        "chosen_predictor": stats[-1]["chosen"],
        "ratio": round(px_rank * 2 / out_len, 4),
    }
    if rank == 0 and world == 1 and not args.no_decode:
        buf = bytes(b)
        t1 = time.perf_counter()
        img = lfm.decode(buf, num_threads=threads)
        dms = (time.perf_counter() - t1) * 1e3
        ref = d_img.cpu().numpy().view(np.uint16)
        line["decode"] = {"ms": round(dms, 1), "Mpixel_per_s": round(px_rank / dms / 1e3, 1),
                          "exact": bool(np.array_equal(img.reshape(ref.shape), ref)),
                          "path": "GPU bzip2 decode + GPU inverse predictor (host libbz2 only for flagged streams, %d threads)" % threads}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(threads=threads)
    if rank == 0:
        print(json.dumps(line), flush=True)
    enc.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
