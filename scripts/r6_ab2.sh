#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r6ab2; mkdir -p $O
export TMPDIR=/tmp
for v in huff16 huff8; do
  LFM_LIB=$PWD/variants/$v/liblfm.so timeout -k 10 300 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "bzip2" > $O/pytest_$v.log 2>&1 || { tail -n 20 $O/pytest_$v.log; exit 1; }
  tail -n 1 $O/pytest_$v.log
done
timeout -k 10 900 scripts/ab_encode.sh $O/ab.jsonl 2 base lib:huff16 lib:huff8 || exit 2
python3 - <<'PY'
import json
for l in open("gpurun_out/r6ab2/ab.jsonl"):
    d=json.loads(l); b=d["bench"]; st=b["stages_ms"]
    print(d["arm"], d["round"], b["value"], b["ms_per_step"], "bwt", st["bz_bwt_ms"], "mtf", st["bz_mtf_ms"], "huf", st["bz_huffman_ms"], "lat", b.get("latency_ms_per_encode"))
PY
LFM_DECODE_TIMING=1 timeout -k 10 300 python scripts/decode_phases.py > $O/dec.log 2>&1; tail -n 12 $O/dec.log
