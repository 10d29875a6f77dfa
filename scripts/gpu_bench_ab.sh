#!/bin/bash
# A/B bench lines (driver-sized: --steps 20 --warmup 5, no decode / host-input /
# CPU baseline) for an env switch: scripts/gpu_bench_ab.sh OUT VAR a,b[,c]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-bab}; VAR=${2:-LFM_HUFF_PACK}; VALS=${3:-32}
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in ${VALS//,/ }; do
  env $VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode --no-host-input > "$OUT/bench_$v.log" 2>&1
  rc=$?; echo "$VAR=$v rc=$rc"; grep -o '"value": [0-9.]*\|"stages_ms": {[^}]*}\|"latency_ms_per_encode": [0-9.]*\|"ok": [a-z]*' "$OUT/bench_$v.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
