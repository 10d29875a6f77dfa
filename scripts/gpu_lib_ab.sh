#!/bin/bash
# Same-box A/B of two builds of liblfm.so (driver-sized bench lines):
# scripts/gpu_lib_ab.sh OUT LIB_A LIB_B [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-libab}; A=$2; B=$3; R=${4:-2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for tag in a b; do
    lib=$A; [ $tag = b ] && lib=$B
    LFM_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --no-host-input --no-config5 --no-small --no-inproc > "$OUT/bench_${tag}_$r.log" 2>&1
    rc=$?; echo "$tag($lib) round $r rc=$rc"; grep -o '"value": [0-9.]*\|"bz_[a-z0-9]*_ms": [0-9.]*\|"latency_ms_per_encode": [0-9.]*\|"ok": [a-z]*\|"kernel_ms": [0-9.]*' "$OUT/bench_${tag}_$r.log" | tr '\n' ' '; echo
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
