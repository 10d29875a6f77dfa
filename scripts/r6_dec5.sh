#!/bin/bash
# decode's first payload upload: SDMA signal wait blocked / active, and the
# runtime copy paths, under the idle probe's patterns
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6dec5; mkdir -p $O
export TMPDIR=/tmp
for arm in base LFM_SDMA_WAIT=1 LFM_DECODE_H2D=2 LFM_DECODE_H2D=1 LFM_SDMA_WAIT=1 base; do
  envs=""; [ "$arm" != base ] && envs="$arm"
  env $envs LFM_DECODE_TIMING=1 timeout -k 10 300 python scripts/decode_idle_probe.py > $O/idle_$arm.log 2>&1 || { tail -n 20 $O/idle_$arm.log; exit 1; }
  echo "== $arm"
  grep -E "ms$" $O/idle_$arm.log | grep -v "decode total\|decode:" | sed -E 's/ \(exact True\)//' | tr '\n' '|' ; echo
  grep -oE "h2d: [0-9]+ bytes, host copies [0-9.]+ ms, waits [0-9.]+ ms( \(first [0-9.]+\))?" $O/idle_$arm.log | awk 'NR%2==1' | sed -E 's/h2d: [0-9]+ bytes, //' | tr '\n' '|'; echo
done
