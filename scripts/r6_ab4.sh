#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ab4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "submit or pipelined or encoder" > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 900 scripts/ab_encode.sh $O/ab.jsonl 3 base "env:LFM_SELECT_AT=2" || exit 2
python3 - <<'PY'
import json
for l in open("gpurun_out/r6ab4/ab.jsonl"):
    d=json.loads(l); b=d["bench"]; st=b["stages_ms"]; rf=b["roofline"]
    print(d["arm"], d["round"], b["value"], b["ms_per_step"], "sel", st["select_ms"], "pred", st["predict_ms"], "kms", rf["kernel_ms"], rf["frac"], "bwt", st["bz_bwt_ms"], "huf", st["bz_huffman_ms"], "lat", b.get("latency_ms_per_encode"))
PY
