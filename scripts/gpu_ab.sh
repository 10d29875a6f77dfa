#!/bin/bash
# GPU parity tests, then A/B bench lines for an env switch (VAR=a,b), then a
# rocprof'd bench with the defaults.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-ab}; VAR=${2:-LFM_CS_XCD}; VALS=${3:-1,0}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
for v in ${VALS//,/ }; do
  env $VAR=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_$v.log" 2>&1
  rc=$?; echo "$VAR=$v rc=$rc"; grep -o '"value": [0-9.]*\|"stages_ms": {[^}]*}\|"decode": {"ms": [0-9.]*' "$OUT/bench_$v.log"
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/bench_prof.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; exit $rc
