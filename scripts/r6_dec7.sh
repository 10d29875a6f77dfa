#!/bin/bash
# decode download: SDMA staged (default) vs runtime copies into the pinned chunks
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6dec7; mkdir -p $O
export TMPDIR=/tmp
for arm in base LFM_DECODE_D2H=1 base LFM_DECODE_D2H=1; do
  envs=""; [ "$arm" != base ] && envs="$arm"
  env $envs LFM_DECODE_TIMING=1 timeout -k 10 300 python scripts/decode_idle_probe.py > $O/idle.log 2>&1 || { tail -n 20 $O/idle.log; exit 1; }
  echo "== $arm"
  grep -E "ms$" $O/idle.log | grep -v "decode total\|decode:" | sed -E 's/ \(exact True\)//' | tr '\n' '|' ; echo
  grep -oE "d2h: [0-9]+ bytes, host copies [0-9.]+ ms, waits [0-9.]+ ms" $O/idle.log | head -n 6 | sed -E 's/d2h: [0-9]+ bytes, //' | tr '\n' '|'; echo
  grep -oE "download [0-9.]+" $O/idle.log | tr '\n' ' '; echo
done
