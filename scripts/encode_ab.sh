#!/bin/bash
# Encode A/B on one box: the bench's timed leg only (config 3, N = 1) under
# several environment settings, each run twice, interleaved.
# usage: scripts/encode_ab.sh OUTFILE "ENV1" "ENV2" ...   ("" = defaults)
set -u -o pipefail
OUT=$1; shift
: > "$OUT"
for rep in 1 2; do
  for e in "$@"; do
    line=$(env $e timeout -k 10 240 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-decode \
           --no-host-input --no-config5 --no-small --no-inproc --config5-host-volumes 0 2>/dev/null | tail -1)
    rc=$?
    echo "{\"env\": \"$e\", \"rep\": $rep, \"rc\": $rc, \"line\": ${line:-null}}" >> "$OUT"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
