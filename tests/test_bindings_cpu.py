"""Binding relink proof: the reference's own MEX sources
(matlabWrapper/{write,read}LFMstack.cpp, readLFMheader.cpp) and JNI source
(src/jni/org_janelia_simview_lfm_LFMJNI.cpp) compile unchanged against
include/lfm and link against liblfm.so.

mex.h and jni.h are MATLAB / JDK headers absent from this image, so
tests/bindings/shim holds declaration-only stand-ins for the few mx* / JNIEnv
names those sources use; they prove source and link compatibility of the
boundary only (nothing is executed).  Every other symbol the linked objects
need must be defined by liblfm.so or the C/C++ runtime.  Reads the sources
from /root/reference (skipped where it is absent, e.g. on the GPU box)."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG, REFERENCE, REPO

SOURCES = ["matlabWrapper/writeLFMstack.cpp", "matlabWrapper/readLFMstack.cpp", "matlabWrapper/readLFMheader.cpp",
           "src/jni/org_janelia_simview_lfm_LFMJNI.cpp"]
SHIM = os.path.join(REPO, "tests", "bindings", "shim")
LIB = os.path.join(PKG, "liblfm.so")


def _nm(path, *flags):
    out = subprocess.run(["nm", "-D", *flags, path], check=True, capture_output=True, text=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if ln.strip()}


@pytest.mark.skipif(not os.path.isdir(REFERENCE) or shutil.which("g++") is None,
                    reason="needs the reference sources and g++")
@pytest.mark.parametrize("src", SOURCES)
def test_reference_binding_compiles_and_links_against_liblfm(tmp_path, src):
    path = os.path.join(REFERENCE, src)
    obj = tmp_path / "b.o"
    so = tmp_path / "b.so"
    # the JNI source includes its own generated header from its directory;
    # klb_imageIO.h / klb_Cwrapper.h / common.h come from include/lfm
    cmd = ["g++", "-std=c++11", "-c", "-fPIC", "-w", "-I", SHIM, "-I", os.path.join(REPO, "include", "lfm"),
           path, "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run(["g++", "-shared", "-o", str(so), str(obj), "-L", PKG, "-llfm"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    undefined = _nm(str(so), "--undefined-only")
    defined = _nm(LIB, "--defined-only")
    foreign = {s for s in undefined if s.startswith(("mx", "mex")) or "JNIEnv" in s or "@" in s
               or s.startswith(("_ITM_", "__gmon_start__", "__cxa_"))}
    missing = sorted(undefined - foreign - defined)
    assert not missing, "symbols the binding needs that liblfm.so does not export: %s" % missing
    # it really binds the boundary (not only the runtime)
    assert any("klb_imageIO" in s or s.startswith(("writeKLB", "readKLB")) for s in undefined - foreign)


def test_boundary_caller_program_links():
    """tests/c/boundary_main (built by __graft_entry__.build) resolves every
    boundary symbol from liblfm.so."""
    exe = os.path.join(REPO, "tests", "c", "boundary_main")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", os.path.dirname(exe)], check=True, capture_output=True)
    undefined = _nm(exe, "--undefined-only")
    needed = {"writeKLBstack", "readKLBstack", "readKLBstackInPlace", "readKLBroiInPlace", "readKLBheader"}
    assert needed <= undefined
    assert needed <= _nm(LIB, "--defined-only")
