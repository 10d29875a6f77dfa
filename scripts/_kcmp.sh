#!/bin/bash
# kernel stats of two library builds on one box: scripts/_kcmp.sh OUT LIB_A LIB_B
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/$1; mkdir -p $OUT
export TMPDIR=/tmp
for tag in a b; do
  lib=$2; [ $tag = b ] && lib=$3
  LFM_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$tag -o k -- python3 bench.py --steps 6 --warmup 3 --no-cpu-baseline --no-host-input --no-decode --no-config5 --no-small --no-inproc > $OUT/$tag.log 2>&1 || exit $?
  grep -o '"value": [0-9.]*' $OUT/$tag.log
done
