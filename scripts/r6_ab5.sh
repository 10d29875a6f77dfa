#!/bin/bash
# hand-written radix chunk sort (variants/rsort) vs rocPRIM merge sort: bzip2
# tests on the variant, then an encode A/B; then the r6_dec3 probes
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ab5; mkdir -p $O
export TMPDIR=/tmp
LFM_LIB=$PWD/variants/rsort/liblfm.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bzip2 or bwt or config3" > $O/pytest_rsort.log 2>&1 || { tail -n 30 $O/pytest_rsort.log; exit 1; }
tail -n 1 $O/pytest_rsort.log
timeout -k 10 900 scripts/ab_encode.sh $O/ab.jsonl 2 base lib:rsort || exit 2
python3 - <<'PY'
import json
for l in open("gpurun_out/r6ab5/ab.jsonl"):
    d=json.loads(l); b=d["bench"]; st=b["stages_ms"]
    print(d["arm"], d["round"], b["value"], b["ms_per_step"], "bwt", st["bz_bwt_ms"], "mtf", st["bz_mtf_ms"], "huf", st["bz_huffman_ms"], "lat", b.get("latency_ms_per_encode"))
PY
scripts/r6_dec3.sh
