#!/bin/bash
# decode downloads on their own stream: runtime copies (default) vs SDMA, config 3 and config 5 legs
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6dec11; mkdir -p $O
export TMPDIR=/tmp
flags="--no-cpu-baseline --no-host-input --no-small --no-inproc --steps 5 --warmup 2"
for r in 1 2; do
  for arm in base LFM_DECODE_D2H=0 LFM_DECODE_D2H=2; do
    envs=""; [ "$arm" != base ] && envs="$arm"
    line=$(env $envs timeout -k 10 300 python3 bench.py $flags 2>>$O/err.log | grep '^{') || { tail -n 20 $O/err.log; exit 1; }
    echo "{\"arm\": \"$arm\", \"round\": $r, \"bench\": $line}" >> $O/ab.jsonl
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print('$arm', $r, d['value'], 'cfg3 decode', d['decode']['runs_ms'], d['decode']['exact'], 'cfg5 decode', d['config5']['decode_runs_ms'], d['config5']['decode_exact'])" "$line"
  done
done
