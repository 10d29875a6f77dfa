#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/reg; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_gpu_full.py -x -q --timeout 300 --timeout-method thread -k "bzip2 or full_size or config4 or manifest or roundtrip" > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
LFM_BZ2_STATS=1 timeout -k 10 300 python bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-host-input --no-decode --no-config5 --no-small --no-inproc 2>&1 | grep "lfm_bzip2 stats" | tail -2
bash scripts/_ab5.sh regab3 exp/liblfm_old.so exp/liblfm_new.so "exp/liblfm_new.so|LFM_TIE_DIRECT=0"
