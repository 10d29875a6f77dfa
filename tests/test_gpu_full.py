"""Full-size byte parity of the BASELINE configs on the GPU.

The oracle's digests (tests/golden/full_size_manifest.json, made by
tests/golden/make_full_size.py with the reference's own bzip2-1.0.6) are
asserted for whole .lfm files produced by the GPU path at the BASELINE sizes:
config 3 (2048 x 2048 x 64, Nnum 15, angle, auto), config 4 (2048 x 2048 x 256,
tiles, auto; one piece and as 8 z-slabs merged, the multi-GPU layout) and one
t-volume of config 5 (4096 x 4096 x 32, video, tiles, auto; encode + decode
round trip)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _full(name):
    return {e["name"]: e for e in json.load(open(os.path.join(GOLDEN, "full_size_manifest.json")))}[name]


def _device_stack(lfmlib, torch, e):
    X, Y, Z = e["xyzct"][:3]
    d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
    lfmlib.synth_device(d, X, Y, Z, e["nnum"], seed=e["seed"])
    torch.cuda.synchronize()
    return d


def _layers(buf, e):
    """SHA-256 of each layer of blocks (one block depth of frames) of a .lfm."""
    h = np.frombuffer(bytes(buf[320:320 + 8 * e["nblocks"]]), dtype="<u8")
    per = e["nblocks"] // len(e["layer_sha256"])
    base = 320 + 8 * e["nblocks"]
    out, prev = [], 0
    for j in range(len(e["layer_sha256"])):
        end = int(h[(j + 1) * per - 1])
        out.append(hashlib.sha256(bytes(buf[base + prev:base + end])).hexdigest())
        prev = end
    return out


def _assert_file(buf, e):
    if hashlib.sha256(buf).hexdigest() != e["sha256"]:
        bad = [j for j, (a, b) in enumerate(zip(_layers(buf, e), e["layer_sha256"])) if a != b]
        pytest.fail("%s: .lfm differs from the oracle (%d vs %d bytes); layers differing: %s"
                    % (e["name"], len(buf), e["size"], bad[:20]))
    assert len(buf) == e["size"]


@pytest.mark.parametrize("name", ["cfg3_2048x2048x64_angle_auto", "cfg4_2048x2048x256_tiles_auto"])
def test_full_size_lfm_sha256(lfmlib, gpu, name):
    e = _full(name)
    d = _device_stack(lfmlib, gpu, e)
    lfmlib.set_family(e["family"])
    enc = lfmlib.Encoder(device=0)
    try:
        buf, st = enc.encode(d, header_version=e["header_version"], nnum=e["nnum"], copy=False)
        assert st["chosen"] == e["chosen"]
        np.testing.assert_allclose(st["entropy"], e["entropy"], rtol=1e-5)
        _assert_file(buf, e)
    finally:
        enc.close()
        lfmlib.set_family("tiles")


def test_config4_eight_slabs_merged(lfmlib, gpu):
    """Config 4 as the 8-GPU layout: 8 z-slabs of 32 frames encoded with the
    predictor selected on frame 0 (forced), joined by lfm_merge_slabs: the
    oracle's one-piece digest."""
    from lfm.shard import forced_request, plan_slabs
    e = _full("cfg4_2048x2048x256_tiles_auto")
    X, Y, Z = e["xyzct"][:3]
    d = _device_stack(lfmlib, gpu, e)
    lfmlib.set_family(e["family"])
    enc = lfmlib.Encoder(device=0)
    try:
        k, _ = lfmlib.select_device(d[0], X, Y, e["nnum"], e["family"])
        assert k == e["chosen"]
        slabs = []
        for z0, dz in plan_slabs(Z, 8, 8):
            b, _ = enc.encode_slab(d[z0:z0 + dz], z0, header_version=forced_request(k), nnum=e["nnum"])
            slabs.append(b)
        _assert_file(lfmlib.merge_slabs(slabs), e)
    finally:
        enc.close()
        lfmlib.set_family("tiles")


def test_config5_volume_roundtrip(lfmlib, gpu):
    """One t-volume of config 5 (4096 x 4096 x 32, video bit, tiles, auto):
    the oracle's bytes, and the GPU decode returns every pixel."""
    e = _full("cfg5v0_4096x4096x32_video_tiles_auto")
    d = _device_stack(lfmlib, gpu, e)
    lfmlib.set_family("tiles")
    enc = lfmlib.Encoder(device=0)
    try:
        buf, st = enc.encode(d, header_version=e["header_version"], nnum=e["nnum"])
        assert st["header_version"] == e["final_header_version"]
        _assert_file(buf, e)
    finally:
        enc.close()
    out = lfmlib.decode(buf)
    assert np.array_equal(out.reshape(d.shape), d.cpu().numpy().view(np.uint16))


@pytest.mark.parametrize("t", [50, 99])
def test_config5_far_volume(lfmlib, gpu, t):
    """t-volume 50 / 99 of the 100-volume config-5 stack (4096 x 4096 x 32,
    video, tiles): coded alone with the predictor chosen on volume 0's frame 0
    (request 8 + k, video bit) its block streams equal the oracle's per-volume
    digest (cfg5far), and the GPU decode returns every pixel.  No synchronise
    between the generator (null stream) and the encode, on purpose: the
    encoder orders its reads of a device input after the null stream's work
    (Encoder::after_caller; without it this test failed now and then)."""
    e = _full("cfg5far_4096x4096x32x1x100_video_tiles_auto")
    X, Y, Z = e["xyzct"][:3]
    want = e["volumes"][str(t)]
    torch = gpu
    d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
    lfmlib.synth_device(d, X, Y, Z, e["nnum"], t_index=t, idx0=t * Z * X * Y, seed=e["seed"])
    lfmlib.set_family("tiles")
    enc = lfmlib.Encoder(device=0)
    try:
        buf, st = enc.encode(d, header_version=0x80 | (8 + e["chosen"]), nnum=e["nnum"])
        assert st["header_version"] == e["final_header_version"]
    finally:
        enc.close()
    base = 320 + 8 * e["nblocks_per_volume"]
    assert len(buf) - base == want["bytes"]
    assert hashlib.sha256(bytes(buf[base:])).hexdigest() == want["sha256"]
    out = lfmlib.decode(buf)
    assert np.array_equal(out.reshape(d.shape), d.cpu().numpy().view(np.uint16))


_CFG5X4_CHILD = r"""
import hashlib, json, os, sys, time
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
import lfm
e = json.loads(sys.argv[2])
path = sys.argv[3]
X, Y, Z, C, Tn = e["xyzct"]
torch.cuda.set_device(0)
d = torch.empty((Z, Y, X), dtype=torch.int16, device="cuda")
img = np.empty((Tn, 1, Z, Y, X), dtype=np.uint16)
for t in range(Tn):  # volume t of the stack: t term and linear index of the SURVEY 8(d) generator
    lfm.synth_device(d, X, Y, Z, e["nnum"], t_index=t, idx0=t * Z * X * Y, seed=e["seed"])
    img[t, 0] = d.cpu().numpy().view(np.uint16)
del d
lfm.set_family("tiles")
t0 = time.perf_counter()
lfm.write_lfm(path, img, predictor_request=0, nnum=e["nnum"], video=1)  # writeLFMstack_c -> writeImage
t_enc = time.perf_counter() - t0
buf = open(path, "rb").read()
nb = e["nblocks"] // Tn
offs = np.frombuffer(buf, dtype="<u8", count=e["nblocks"], offset=320)
base, prev, vols = 320 + 8 * e["nblocks"], 0, []
for t in range(Tn):
    end = int(offs[(t + 1) * nb - 1])
    vols.append(hashlib.sha256(buf[base + prev:base + end]).hexdigest())
    prev = end
t0 = time.perf_counter()
back, hv, nn = lfm.read_lfm(path)  # readLFMstack_c -> readImageFull
t_dec = time.perf_counter() - t0
print(json.dumps({"sha256": hashlib.sha256(buf).hexdigest(), "size": len(buf), "volume_sha256": vols,
                  "header_version": hv, "exact": bool(np.array_equal(back, img)),
                  "encode_s": t_enc, "decode_s": t_dec, "devices": lfm.get_devices()}))
"""


@pytest.mark.timeout(600)
def test_config5_four_volumes_t_sharded_writer(lfmlib, gpu, tmp_path):
    """Config 5 at full frame size, four t-volumes (4096 x 4096 x 32 x 1 x 4,
    video, tiles, auto) through the drop-in writer: writeLFMstack_c ->
    klb_imageIO::writeImage farms the t-axis over LFM_GPUS=0,0,0,0 (four
    workers on the test box's one GPU, lfm_multigpu.cpp) and the file equals
    the oracle's (whole-file and per-volume SHA-256, full_size_manifest.json
    cfg5x4); readLFMstack_c -> readImageFull returns every pixel.  Runs in a
    child process (its own pooled encoders and workspace budget)."""
    import subprocess
    import sys
    from conftest import PKG
    e = _full("cfg5x4_4096x4096x32x1x4_video_tiles_auto")
    env = dict(os.environ, LFM_GPUS="0,0,0,0", LFM_BZ2_GPU_BUDGET_MB="6144")
    r = subprocess.run([sys.executable, "-c", _CFG5X4_CHILD, PKG, json.dumps(e), str(tmp_path / "cfg5x4.lfm")],
                       env=env, capture_output=True, text=True, timeout=560)
    assert r.returncode == 0, r.stderr[-3000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert got["devices"] == [0, 0, 0, 0]
    assert got["volume_sha256"] == e["volume_sha256"]
    assert got["sha256"] == e["sha256"] and got["size"] == e["size"]
    assert got["header_version"] == e["final_header_version"]
    assert got["exact"]
    print("cfg5x4: encode %.2f s, decode %.2f s" % (got["encode_s"], got["decode_s"]))
