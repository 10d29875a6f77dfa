#!/bin/bash
# Encode-only bench A/B on one box: scripts/ab_encode.sh OUT ROUNDS LIB_OR_ENV...
# each arm: "lib:<variant dir under variants/>", "env:VAR=VALUE", or "base";
# the arms alternate ROUNDS times; one JSON line per run goes to OUT.
out=$1; rounds=$2; shift 2
flags="--no-cpu-baseline --no-decode --no-host-input --no-config5 --no-small --no-inproc --steps 10 --warmup 3"
for r in $(seq 1 $rounds); do
  for arm in "$@"; do
    case $arm in
      lib:*) envs="LFM_LIB=$GRAFT_REPO_ROOT/variants/${arm#lib:}/liblfm.so" ;;
      env:*) envs="${arm#env:}" ;;
      *) envs="" ;;
    esac
    line=$(env $envs timeout -k 10 240 python3 bench.py $flags 2>>${out%.jsonl}.err | grep '^{') || exit 1
    echo "{\"arm\": \"$arm\", \"round\": $r, \"bench\": $line}" >> $out
    echo "$arm $r done"
  done
done
