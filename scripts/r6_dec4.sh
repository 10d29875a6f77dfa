#!/bin/bash
# decode: destination prefault off / during the first upload / after it
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6dec4; mkdir -p $O
export TMPDIR=/tmp
for m in 1 2 0 2 1; do
  LFM_DECODE_PREFAULT=$m LFM_DECODE_TIMING=1 timeout -k 10 300 python scripts/decode_idle_probe.py > $O/idle_$m.log 2>&1 || { tail -n 20 $O/idle_$m.log; exit 1; }
  echo "== prefault $m"
  grep -E "ms$" $O/idle_$m.log | grep -v "decode total" | tr '\n' '|' ; echo
  grep -oE "uploaded 0@[0-9.]+|prefault-done 0@[0-9.]+|dl-start 0@[0-9.]+" $O/idle_$m.log | tr '\n' ' '; echo
done
timeout -k 10 300 python -u -m pytest tests/test_gpu.py tests/test_boundary_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "decode or unpredict or boundary" > $O/pytest.log 2>&1; rc=$?; tail -n 2 $O/pytest.log; exit $rc
