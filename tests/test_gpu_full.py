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
