#!/bin/bash
# Round-6 GPU session: full GPU tests, smoke, bench, rocprof kernel trace of
# the bench.  Each step under its own time limit; stops at the first step
# that crashes or times out (rc other than 0 / 1).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r6}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -n 4 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return $rc
}
[ "${TESTS:-1}" = "1" ] && step pytest_gpu 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_ARGS:-}
[ "${SMOKE:-1}" = "1" ] && step smoke 300 python __graft_entry__.py smoke
[ "${BENCH:-1}" = "1" ] && step bench 600 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-host-input
fi
echo ALL_DONE
