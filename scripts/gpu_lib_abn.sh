#!/bin/bash
# Same-box comparison of several liblfm.so builds (driver-sized bench lines,
# encode only), rounds interleaved: scripts/gpu_lib_abn.sh OUT ROUNDS LIB...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-libabn}; R=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  i=0
  for lib in "$@"; do
    LFM_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --no-host-input --no-config5 --no-small --no-inproc > "$OUT/bench_${i}_$r.log" 2>&1
    rc=$?; echo "[$i] $lib round $r rc=$rc"; grep -o '"value": [0-9.]*\|"bz_[a-z0-9]*_ms": [0-9.]*\|"latency_ms_per_encode": [0-9.]*\|"ok": [a-z]*\|"kernel_ms": [0-9.]*' "$OUT/bench_${i}_$r.log" | tr '\n' ' '; echo
    [ $rc -ne 0 ] && exit $rc
    i=$((i + 1))
  done
done
exit 0
