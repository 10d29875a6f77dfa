#!/bin/bash
# decode A/B on one box: round-5 library vs this tree, prefault on / off
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ab3; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "decode or roi or read" > $O/pytest_dec.log 2>&1 || { tail -n 30 $O/pytest_dec.log; exit 1; }
tail -n 1 $O/pytest_dec.log
for r in 1 2; do
  for arm in base r5 noprefault; do
    case $arm in
      base) envs="" ;;
      r5) envs="LFM_LIB=$PWD/variants/r5/liblfm.so" ;;
      noprefault) envs="LFM_DECODE_PREFAULT=0" ;;
    esac
    env LFM_DECODE_TIMING=1 $envs timeout -k 10 300 python scripts/decode_phases.py > $O/dec_${arm}_$r.log 2>&1 || { tail -n 20 $O/dec_${arm}_$r.log; exit 2; }
    echo "$arm $r: $(grep -E '^decode [0-9]' $O/dec_${arm}_$r.log | tr '\n' ' ')"
    grep "chunks of" $O/dec_${arm}_$r.log | tail -n 1
  done
done
