#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ab1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bzip2 or lfm_manifest or full" > $O/pytest_bz.log 2>&1; rc=$?
tail -n 3 $O/pytest_bz.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 scripts/ab_encode.sh $O/ab.jsonl 2 base lib:noswz "env:GPU_MAX_HW_QUEUES=8" "env:GPU_MAX_HW_QUEUES=8 LFM_BZ2_SLOTS=3"
python3 - <<'PY'
import json
for l in open("gpurun_out/r6ab1/ab.jsonl"):
    d=json.loads(l); b=d["bench"]; st=b["stages_ms"]
    print(d["arm"], d["round"], b["value"], b["ms_per_step"], "bwt", st["bz_bwt_ms"], "mtf", st["bz_mtf_ms"], "huf", st["bz_huffman_ms"], "lat", b.get("latency_ms_per_encode"))
PY
