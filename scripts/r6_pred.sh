#!/bin/bash
# predictor parity tests, then standalone roofline A/B of the predictor kernels
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r6pred}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "spatial_stack or golden_predictor or fast_kernel or video_frame_pairs or candidates or z0_offset" > $O/pytest_pred.log 2>&1; rc=$?
tail -n 3 $O/pytest_pred.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for arm in "" "LFM_PRED_RW=0" "LFM_PRED_RW_PIECES=4" "LFM_PRED_RW_PIECES=16"; do
    env $arm timeout -k 10 200 python scripts/pred_standalone.py "${arm:-rw}" >> $O/standalone.jsonl 2>> $O/standalone.err || exit 3
  done
done
python3 - <<PY
import json
for l in open("$O/standalone.jsonl"):
    d=json.loads(l)
    print(d["label"], "warm", d["warm"]["kernel_ms_median"], d["warm"]["frac"], "flushed", d["flushed"]["kernel_ms_median"], d["flushed"]["frac"], "copy", d["copies"]["torch_add"]["warm"]["frac"])
PY
