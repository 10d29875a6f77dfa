#!/bin/bash
# usage: scripts/sweep.sh OUT "ENV=.. ENV2=.." "ENV=.." ...  -- bench once per env setting
set -u
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
i=0
for envs in "$@"; do
  i=$((i+1))
  env $envs timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/b$i.log" 2>&1
  rc=$?
  echo "[$envs] rc=$rc $(grep -o '"value": [0-9.]*' "$OUT/b$i.log") $(grep -o '"stages_ms": {[^}]*}' "$OUT/b$i.log")"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/b$i.log"; exit $rc; fi
done
