"""The drop-in boundary as a C/C++ caller uses it, on the GPU: tests/c/boundary_main
(linked against liblfm.so, reference header names) runs writeKLBstack (uint16,
auto-select, Nnum 13), readKLBstack (+ free), readKLBstackInPlace, the MEX
klb_imageIO member sequence, readKLBroiInPlace and readKLBheader; its .lfm
files are compared byte for byte with the oracle (reference bzip2-1.0.6) and
the committed fixtures."""
import hashlib
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO

pytestmark = pytest.mark.gpu
EXE = os.path.join(REPO, "tests", "c", "boundary_main")


def _run(tmp_path, img, request, video):
    Z, Y, X = img.shape
    raw = tmp_path / "in.u16"
    raw.write_bytes(np.ascontiguousarray(img, dtype="<u2").tobytes())
    assert os.path.exists(EXE), "tests/c/boundary_main not built (run __graft_entry__.build())"
    env = dict(os.environ, LFM_PREDICTOR_WAY="0")
    r = subprocess.run([EXE, str(raw), str(X), str(Y), str(Z), str(tmp_path), str(request), str(video)],
                       capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "timed out" not in r.stderr, r.stderr  # (no inverse-predictor hand-over gave up)
    return (tmp_path / "klb.lfm").read_bytes(), (tmp_path / "mex.lfm").read_bytes()


def test_boundary_program_on_reference_img_tif(oracle, gpu, tmp_path):
    """The reference's own testData/img.tif stack (29 x 151 x 101): the MEX
    sequence with an auto request and the video bit gives the committed
    fixture; writeKLBstack gives the oracle's auto-select bytes."""
    img = np.load(os.path.join(GOLDEN, "img_tif.npz"))["img"]
    klb, mex = _run(tmp_path, img, 0, 1)
    man = {e["name"]: e for e in json.load(open(os.path.join(GOLDEN, "lfm_manifest.json")))}
    e = man["imgtif_stack_auto_video"]
    assert mex == open(os.path.join(GOLDEN, e["file"]), "rb").read()
    assert hashlib.sha256(mex).hexdigest() == e["sha256"]
    meta = b"boundary_main"
    assert klb == oracle.encode(img[None, None], header_version=0, nnum=13, family="tiles",
                                pixel_size=[1.0] * 5, metadata=meta)


def test_boundary_program_synthetic_forced(oracle, gpu, tmp_path):
    """A synthetic light-field stack (several blocks in x, y and z) with a
    forced predictor request through the MEX sequence (request 8 + 5)."""
    img = oracle.synthetic_lf(520, 300, Z=12, T=13, seed=0x4C464D09)[0, 0]
    klb, mex = _run(tmp_path, img, 8 + 5, 0)
    assert mex == oracle.encode(img[None, None], header_version=8 + 5, nnum=13, family="tiles",
                                pixel_size=[1.0] * 5)
    assert klb == oracle.encode(img[None, None], header_version=0, nnum=13, family="tiles",
                                pixel_size=[1.0] * 5, metadata=b"boundary_main")
