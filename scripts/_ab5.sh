#!/bin/bash
# same-box A/B over "LIB|ENV..." items: scripts/_ab5.sh OUT ITEM...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; shift; mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2; do
  for it in "$@"; do
    lib=${it%%|*}; envs=""; [ "$it" != "$lib" ] && envs=${it#*|}
    env LFM_LIB=$lib $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --no-host-input --no-config5 --no-small --no-inproc > $OUT/b.log 2>&1
    rc=$?; echo "$it r$r rc=$rc $(grep -o '"value": [0-9.]*\|"kernel_ms": [0-9.]*\|"bz_bwt_ms": [0-9.]*\|"bz_huffman_ms": [0-9.]*\|"latency_ms_per_encode": [0-9.]*\|"ok": [a-z]*' $OUT/b.log | tr '\n' ' ')"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
