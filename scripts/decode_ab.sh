#!/bin/bash
# Decode A/B on one box: decode_phases.py under several env settings
# (LFM_DECODE_TIMING phase times), then one rocprofv3 kernel-stats run.
# usage: bash scripts/decode_ab.sh OUTDIR "ENV1" "ENV2" ...   (ENV: "A=1 B=2")
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-decode_ab}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp LFM_DECODE_TIMING=1
i=0
for cfg in "$@"; do
    echo "=== [$i] $cfg" | tee -a "$OUT/ab.log"
    env $cfg timeout -k 10 240 python scripts/decode_phases.py >> "$OUT/ab.log" 2>&1
    rc=$?
    echo "=== [$i] rc=$rc" | tee -a "$OUT/ab.log"
    grep -E "phase (upload|bunzip2|unpredict|download)|^decode [0-9]" "$OUT/ab.log" | tail -15
    if [ $rc -ne 0 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
    i=$((i + 1))
done
if [ -n "${PROF_ENV:-}" ]; then
    env $PROF_ENV timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o dec -- python scripts/decode_phases.py > "$OUT/prof.log" 2>&1 || exit $?
fi
echo ALL_DONE
