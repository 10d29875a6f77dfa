#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6dec3; mkdir -p $O
export TMPDIR=/tmp
LFM_DECODE_TIMING=1 timeout -k 10 300 python scripts/decode_idle_probe.py > $O/idle.log 2>&1; rc=$?
grep -E "ms$|timeline" $O/idle.log | sed -E 's/(timeline: [^u]*)uploaded 0@([0-9.]+).*/\1 uploaded0@\2/' | cut -c1-200
exit $rc
