#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace.
# Stops at the first step that crashes / times out (exit 124, 134, 137, 139 or
# any rc other than 0/1 from pytest); assertion failures (rc 1) do not stop it.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "=== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -5 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return $rc
}
rocm-smi --showproductname > "$OUT/rocm_smi.log" 2>&1 || true
[ "${TESTS:-1}" = "1" ] && step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
[ "${TESTS:-1}" = "1" ] && step smoke 300 python __graft_entry__.py smoke
[ "${BENCH:-1}" = "1" ] && step bench 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup ${BENCH_WARMUP:-5}
if [ "${PROFILE:-1}" = "1" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-host-input
fi
echo ALL_DONE
