"""In-process multi-GPU writer: klb_imageIO::writeImage /
writeKLBstack / lfm_encoder_encode_multi farm block-layer ranges over the
device list, one host thread each, and append them in order.  On a one-GPU
box several workers map onto device 0 (lfm_set_devices([0, 0, ...]) or
LFM_GPUS=0,0,...): every worker is its own encoder with its own buffers, so
the path is the same as on an 8-GPU node.  Output must equal the one-device
encode and the oracle byte for byte."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture
def workers(lfmlib):
    yield lambda n: lfmlib.set_devices([0] * n)
    lfmlib.set_devices(None)
    lfmlib.release_encoders()
    lfmlib.set_family("tiles")


def test_multi_config3_full_size(lfmlib, gpu, workers):
    """Config 3 (2048 x 2048 x 64, angle, auto) from a host buffer on 4
    workers (16-frame slabs): the oracle's full-size digest."""
    e = {x["name"]: x for x in json.load(open(os.path.join(GOLDEN, "full_size_manifest.json")))}[
        "cfg3_2048x2048x64_angle_auto"]
    X, Y, Z = e["xyzct"][:3]
    d = gpu.empty((Z, Y, X), dtype=gpu.int16, device="cuda")
    lfmlib.synth_device(d, X, Y, Z, e["nnum"], seed=e["seed"])
    img = d.cpu().numpy().view(np.uint16)
    del d
    lfmlib.set_family("angle")
    workers(4)
    enc = lfmlib.Encoder(device=0)
    buf, st = enc.encode_multi(img, header_version=0, nnum=e["nnum"], copy=False)
    assert st["chosen"] == e["chosen"]
    assert hashlib.sha256(buf).hexdigest() == e["sha256"]
    enc.close()


@pytest.mark.parametrize("n", [2, 3, 5])
def test_multi_video_slabs_match_oracle(lfmlib, oracle, gpu, workers, n):
    """Video tiles stack with a 3-deep block: slabs start at odd frames (the
    previous raw frame comes from the host image) and the last slab is
    shallower than a block (the level stays the whole stack's)."""
    img = oracle.synthetic_lf(200, 96, Z=20, T=13, seed=0x4C464D0A)
    bs = [64, 32, 3, 1, 1]
    want = oracle.encode(img, header_version=0x80, nnum=13, family="tiles", block_size=bs)
    workers(n)
    enc = lfmlib.Encoder(device=0)
    got, st = enc.encode_multi(img, header_version=0x80, nnum=13, block_size=bs)
    enc.close()
    assert got == want


def test_multi_default_blocks_partial_last_layer(lfmlib, oracle, gpu, workers):
    """Default 96 x 96 x 8 blocks, 20 frames on 3 workers (8, 8, 4 frames):
    the 4-frame slab codes at the 8-frame block's bzip2 level."""
    img = oracle.synthetic_lf(300, 200, Z=20, T=15, seed=0x4C464D0B)
    want = oracle.encode(img, header_version=0, nnum=15, family="tiles")
    workers(3)
    enc = lfmlib.Encoder(device=0)
    got, _ = enc.encode_multi(img, header_version=0, nnum=15)
    enc.close()
    assert got == want


def test_multi_ranges_of_t_and_c(lfmlib, oracle, gpu, workers):
    """5-D stacks shard by t (or c when t = 1); one predictor chosen on
    volume (0, 0), forced for every range."""
    workers(2)
    enc = lfmlib.Encoder(device=0)
    for shape in ((3, 2), (1, 3)):
        img = oracle.synthetic_lf(128, 100, Z=5, C=shape[1], Tn=shape[0], T=13, seed=0x4C464D0C)
        want = oracle.encode(img, header_version=0x80, nnum=13, family="tiles", block_size=[64, 64, 2, 1, 1])
        got, _ = enc.encode_multi(img, header_version=0x80, nnum=13, block_size=[64, 64, 2, 1, 1])
        assert got == want, shape
    enc.close()


def test_write_klb_stack_uses_lfm_gpus(lfmlib, oracle, gpu, tmp_path, monkeypatch):
    """writeKLBstack (reference C ABI: auto-select, Nnum 13) with LFM_GPUS
    naming three workers: the oracle's bytes."""
    img = oracle.synthetic_lf(256, 192, Z=24, T=13, seed=0x4C464D0D)
    monkeypatch.setenv("LFM_GPUS", "0,0,0")
    try:
        assert lfmlib.get_devices() == [0, 0, 0]
        p = tmp_path / "w.lfm"
        lfmlib.write_klb(p, img)
    finally:
        monkeypatch.delenv("LFM_GPUS")
        lfmlib.release_encoders()
    assert p.read_bytes() == oracle.encode(img, header_version=0, nnum=13, family="tiles")


@pytest.mark.timeout(420)
def test_bench_two_ranks_one_shared_lfm(gpu, tmp_path):
    """`python bench.py --gpus 2` (no launcher: bench.py starts the two ranks
    itself, torchrun as a child; gloo stands in for RCCL, both ranks on device
    0, 16 frames per rank): every rank encodes its slab with the product
    encoder, the slab sizes are all_gathered and every rank places its blocks
    into one shared .lfm; rank 0 checks it against the oracle's per-layer
    digests (`verified`).  Then rank 0 runs the `inproc` leg -- the drop-in
    writer on config 4 over the N ranks' devices (here two workers on the one
    GPU) -- while the other rank waits on the host: both encodes give the
    oracle's cfg4 bytes."""
    import subprocess
    import sys
    from conftest import REPO
    env = dict(os.environ, LFM_BENCH_BACKEND="gloo", OMP_NUM_THREADS="4", LFM_BZ2_GPU_BUDGET_MB="8192")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--frames", "16", "--steps", "2",
           "--warmup", "1", "--no-decode", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["verified"]["ok"], line
    legs = line["inproc"]
    assert legs["gpus_1"]["verified"] is True, legs
    assert legs["workers_2"]["verified"] is True and legs["workers_2"]["devices"] == [0, 0], legs


@pytest.mark.timeout(320)
def test_bench_inproc_leg_four_workers(gpu, tmp_path):
    """bench.py's `inproc` leg -- the drop-in writer (lfm_encoder_encode_multi,
    what klb_imageIO::writeImage runs) on config 4 from host memory -- with
    four workers mapped onto the one GPU (LFM_BENCH_INPROC=0,0,0,0): both the
    one-device and the four-worker encodes give the oracle's cfg4 bytes, so
    `--gpus 1` on an 8-GPU node times the same code path over 8 devices."""
    import subprocess
    import sys
    from conftest import REPO
    env = dict(os.environ, LFM_BENCH_INPROC="0,0,0,0", LFM_BZ2_GPU_BUDGET_MB="8192")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "1", "--warmup", "1", "--frames", "16",
           "--no-decode", "--no-cpu-baseline", "--no-host-input", "--no-config5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    legs = line["inproc"]
    assert legs["gpus_1"]["verified"] is True, legs
    assert legs["workers_4"]["verified"] is True and legs["workers_4"]["devices"] == [0, 0, 0, 0], legs
