#!/bin/bash
# decode's slow first upload: a timed 64 KiB SDMA copy at decode entry, and switches
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6dec6; mkdir -p $O
export TMPDIR=/tmp
for arm in LFM_DECODE_DMA_PROBE=1 "LFM_DECODE_DMA_PROBE=1 LFM_DECODE_SLACK=0" LFM_DECODE_KEEP=0; do
  tag=$(echo $arm | tr ' =' '_-')
  env $arm LFM_DECODE_TIMING=1 timeout -k 10 300 python scripts/decode_idle_probe.py > $O/idle_$tag.log 2>&1 || { tail -n 20 $O/idle_$tag.log; exit 1; }
  echo "== $arm"
  grep -E "ms$" $O/idle_$tag.log | grep -v "decode total\|decode:" | sed -E 's/ \(exact True\)//' | tr '\n' '|' ; echo
  grep -oE "dma probe: 64 KiB upload [0-9.]+ ms" $O/idle_$tag.log | sed -E 's/dma probe: 64 KiB upload //' | tr '\n' '|'; echo
  grep -oE "h2d: [0-9]+ bytes, host copies [0-9.]+ ms, waits [0-9.]+ ms( \(first [0-9.]+\))?" $O/idle_$tag.log | grep -v "h2d: 65536" | awk 'NR%2==1' | sed -E 's/h2d: [0-9]+ bytes, host copies [0-9.]+ ms, //' | tr '\n' '|'; echo
done
