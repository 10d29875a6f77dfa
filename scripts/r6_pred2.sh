#!/bin/bash
# predictor launch shape A/B (angle, config 3): prefetch depth and compute waves
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6pred2; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for v in base pd2 pd4 pd5 ncw8; do
    envs=""; [ "$v" != base ] && envs="LFM_LIB=$PWD/variants/$v/liblfm.so"
    env $envs timeout -k 10 120 python scripts/pred_standalone.py $v >> $O/std.jsonl 2>> $O/std.err || { tail -n 20 $O/std.err; exit 1; }
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r6pred2/std.jsonl"):
    d=json.loads(l)
    print(d["label"], "warm", d["warm"]["kernel_ms_median"], d["warm"]["frac"], "flushed", d["flushed"]["kernel_ms_median"], d["flushed"]["frac"], "add", d["copies"]["torch_add"]["warm"]["frac"], d["copies"]["torch_add"]["flushed"]["frac"])
PY
