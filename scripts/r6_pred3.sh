#!/bin/bash
# predictor: two rows per compute wave and step (RPW 2, prefetch 1 or 2 steps) vs the kept shape
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6pred3; mkdir -p $O
export TMPDIR=/tmp
for v in rpw2pd1 rpw2pd2; do
  LFM_LIB=$PWD/variants/$v/liblfm.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "predict or config3 or vec" > $O/pytest_$v.log 2>&1 || { tail -n 20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -n 1 $O/pytest_$v.log)"
done
for r in 1 2; do
  for v in base rpw2pd1 rpw2pd2; do
    envs=""; [ "$v" != base ] && envs="LFM_LIB=$PWD/variants/$v/liblfm.so"
    env $envs timeout -k 10 120 python scripts/pred_standalone.py $v >> $O/std.jsonl 2>> $O/std.err || { tail -n 20 $O/std.err; exit 1; }
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r6pred3/std.jsonl"):
    d=json.loads(l)
    print(d["label"], "warm", d["warm"]["kernel_ms_median"], d["warm"]["frac"], "flushed", d["flushed"]["kernel_ms_median"], d["flushed"]["frac"], "add", d["copies"]["torch_add"]["warm"]["frac"])
PY
