#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/dec; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "decode or bunzip2 or roundtrip" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash scripts/decode_ab.sh dec_ab "LFM_BZD_VALU=0" "LFM_BZD_VALU=1" "LFM_BZD_VALU=0" "LFM_BZD_VALU=1"
