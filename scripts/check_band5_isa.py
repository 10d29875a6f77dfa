"""Build-time check of the inverse predictor's hand-counted release wait
(ADVICE r03): unpredict_band5 publishes a band's progress after
`s_waitcnt vmcnt(2)` (vmcnt(3) on temporal frames), counting on exactly the
round's group loads having been issued after the round's last pixel store.
vmcnt counts a wave's vector memory operations in issue order, so the wait
proves the store complete only if at least N vector memory instructions
follow that store before the wait.  This compiles unpredict_band5 for one
predictor of each family (device assembly), finds every hand-written
`s_waitcnt vmcnt(N)` with N > 0 (inline asm between ;;#ASMSTART / ;;#ASMEND)
and checks that rule against the instructions the compiler actually placed.

python scripts/check_band5_isa.py [--keep-asm PATH]   (exit 1 on a violation)"""
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "lightfieldmicroscopy_pc-bzip2_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SRC = r"""
#define LFM_UNPREDICT_NO_ENTRY
#include "lfm_unpredict.hip"
template __global__ void lfm::unpredict_band5<0, 4>(lfm::UnFrames, int*, int, int);
template __global__ void lfm::unpredict_band5<1, 5>(lfm::UnFrames, int*, int, int);
template __global__ void lfm::unpredict_band5<2, 7>(lfm::UnFrames, int*, int, int);
"""

VMEM = re.compile(r"^\s+(buffer_|global_|flat_)(load|store|atomic)")
STORE = re.compile(r"^\s+buffer_store_dwordx4\b")


def compile_asm(out):
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "band5_check.hip")
        open(src, "w").write(SRC)
        cmd = [HIPCC, "-O3", "-std=c++17", "-I", os.path.join(REPO, "include", "lfm"), "-I", CSRC,
               "--offload-arch=gfx950", "--offload-device-only", "-S", src, "-o", out]
        subprocess.run(cmd, check=True, capture_output=True)


def check(asm_path):
    """[(kernel, wait N, vector memory ops issued after the second-to-last
    pixel store on the loop's back edge)] for every hand-written wait.

    The wait sits at the top of the band's 32-step loop; it must find the
    stores of every round but the last complete: they are complete when at
    least N vector memory instructions were issued after the second-to-last
    round's pixel store (the last round's store and its group loads).  The
    path to the wait is the loop's back edge: scan backward from the branch
    that closes the innermost loop around the wait."""
    lines = open(asm_path).read().splitlines()
    labels = {}
    for i, ln in enumerate(lines):
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            labels[m.group(1)] = i
    found, kernel, inside = [], None, False
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\S*unpredict_band5\S*):", ln)
        if m:
            kernel = m.group(1)
        elif re.match(r"^_Z\S*:", ln):
            kernel = None
        if ln.strip() == ";;#ASMSTART":
            inside = True
            continue
        if ln.strip() == ";;#ASMEND":
            inside = False
            continue
        w = re.match(r"^\s+s_waitcnt vmcnt\((\d+)\)\s*$", ln)
        if not (inside and w and kernel) or int(w.group(1)) == 0:
            continue
        n = int(w.group(1))
        latch = None
        for j in range(i + 1, len(lines)):
            if re.match(r"^_Z\S*:", lines[j]) or lines[j].startswith(".Lfunc_end"):
                break
            b = re.match(r"^\s+s_(?:c)?branch\S*\s+(\.LBB\S+)", lines[j])
            if b and labels.get(b.group(1), 1 << 30) <= i:
                latch = j
                break
        ops, stores = 0, 0
        if latch is not None:
            for j in range(latch, i, -1):
                if VMEM.match(lines[j]):
                    ops += 1
                if STORE.match(lines[j]):
                    stores += 1
                    if stores == 2:
                        ops -= 1  # the second-to-last store itself does not count
                        break
        found.append((kernel, n, ops if stores == 2 else -1))
    return found


def main():
    keep = sys.argv[sys.argv.index("--keep-asm") + 1] if "--keep-asm" in sys.argv else None
    with tempfile.TemporaryDirectory() as d:
        asm = keep or os.path.join(d, "band5.s")
        compile_asm(asm)
        res = check(asm)
    bad = [r for r in res if r[2] < r[1]]
    for k, n, ops in res:
        print("%s vmcnt(%d): %d vector memory ops after the second-to-last pixel store%s" % (k, n, ops,
                                                                                  "" if ops >= n else "  VIOLATION"))
    if not res:
        print("no hand-written waits found")
        return 1
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
