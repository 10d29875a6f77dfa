#!/bin/bash
# mtf_win match masks by ballots (default build) vs LDS atomicOr (variants/mtfatomic)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ab7; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_gpu_full.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bzip2 or bwt or mtf or config3 or config4 or config5" > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 1 $O/pytest.log
timeout -k 10 900 scripts/ab_encode.sh $O/ab.jsonl 3 base lib:mtfatomic || exit 2
python3 - <<'PY'
import json
for l in open("gpurun_out/r6ab7/ab.jsonl"):
    d=json.loads(l); b=d["bench"]; st=b["stages_ms"]
    print(d["arm"], d["round"], b["value"], b["ms_per_step"], "bwt", st["bz_bwt_ms"], "mtf", st["bz_mtf_ms"], "huf", st["bz_huffman_ms"], "lat", b.get("latency_ms_per_encode"))
PY
