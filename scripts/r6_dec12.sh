#!/bin/bash
# bench decode leg: 2 slots / 2 chunks (default) vs 3 slots with 3 or 4 chunks
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6dec12; mkdir -p $O
export TMPDIR=/tmp
flags="--no-cpu-baseline --no-host-input --no-config5 --no-small --no-inproc --steps 5 --warmup 2"
for r in 1 2; do
  for arm in base "LFM_DECODE_SLOTS=3 LFM_DECODE_CHUNK_BLOCKS=1300" "LFM_DECODE_SLOTS=3 LFM_DECODE_CHUNK_BLOCKS=968"; do
    envs=""; [ "$arm" != base ] && envs="$arm"
    line=$(env $envs timeout -k 10 240 python3 bench.py $flags 2>>$O/err.log | grep '^{') || { tail -n 20 $O/err.log; exit 1; }
    echo "{\"arm\": \"$arm\", \"round\": $r, \"bench\": $line}" >> $O/ab.jsonl
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('$arm', $r, d['value'], d['decode'])" "$line"
  done
done
