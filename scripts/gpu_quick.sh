#!/bin/bash
# Quick GPU iteration: GPU parity tests, then one rocprof'd bench (no CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench.log" 2>&1
rc2=$?; grep '"metric"' "$OUT/bench.log" | cut -c1-400; echo "bench rc=$rc2"
exit $rc
