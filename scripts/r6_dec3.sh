#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6dec3; mkdir -p $O
export TMPDIR=/tmp
LFM_LIB=$PWD/variants/ent1024/liblfm.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "entrop or select" > $O/pytest_ent.log 2>&1 || { tail -n 20 $O/pytest_ent.log; exit 1; }
tail -n 1 $O/pytest_ent.log
for r in 1 2 3; do
  timeout -k 10 120 python scripts/select_probe.py base
  LFM_LIB=$PWD/variants/ent1024/liblfm.so timeout -k 10 120 python scripts/select_probe.py ent1024
done
LFM_DECODE_TIMING=1 timeout -k 10 300 python scripts/decode_idle_probe.py > $O/idle.log 2>&1; rc=$?
grep -E "ms$|timeline" $O/idle.log | grep -v "decode total" | sed -E 's/decode timeline: .*uploaded 0@([0-9.]+).*/  first upload done @\1 ms/'
exit $rc
