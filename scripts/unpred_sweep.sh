#!/bin/bash
# Inverse-predictor band5 hand-over knobs, one box: unpred_probe.py per env.
# usage: bash scripts/unpred_sweep.sh OUTDIR "ENV1" "ENV2" ...
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-usweep}; shift
mkdir -p "$OUT"
i=0
for cfg in "$@"; do
    echo "=== [$i] $cfg"
    env $cfg timeout -k 10 120 python scripts/unpred_probe.py > "$OUT/probe_$i.log" 2>&1
    rc=$?
    grep shape "$OUT/probe_$i.log" | tr '\n' ' ' | sed 's/"xcu": "1"//g'; echo
    if [ $rc -ne 0 ]; then echo "stopping (rc=$rc)"; tail -5 "$OUT/probe_$i.log"; exit $rc; fi
    i=$((i + 1))
done
