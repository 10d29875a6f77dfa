#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6dec2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "decode or roi or read or unpredict" > $O/pytest_dec.log 2>&1 || { tail -n 30 $O/pytest_dec.log; exit 1; }
tail -n 1 $O/pytest_dec.log
for r in 1 2; do
  for arm in slack sync closed; do
    envs="LFM_DECODE_SLACK=1"; [ $arm = sync ] && envs="LFM_DECODE_SLACK=0"; [ $arm = closed ] && envs="CLOSE_ENC=1"
    env $envs LFM_DECODE_TIMING=1 timeout -k 10 300 python scripts/decode_phases.py > $O/dec_${arm}_$r.log 2>&1 || { tail -n 20 $O/dec_${arm}_$r.log; exit 2; }
    echo "$arm $r: $(grep -E '^decode [0-9]' $O/dec_${arm}_$r.log | cut -d, -f1 | tr '\n' ' ')"
    grep "timeline" $O/dec_${arm}_$r.log | tail -n 1 | cut -c1-420
  done
done
