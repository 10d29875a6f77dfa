#!/bin/bash
# same-box A/B over several library builds: scripts/_ab4.sh OUT LIB...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for lib in "$@"; do
    LFM_LIB=$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --no-host-input --no-config5 --no-small --no-inproc > $OUT/b.log 2>&1
    rc=$?; echo "$lib r$r rc=$rc $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"select_ms": [0-9.]*\|"bz_emit_ms": [0-9.]*\|"latency_ms_per_encode": [0-9.]*\|"ok": [a-z]*' $OUT/b.log | tr '\n' ' ')"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
