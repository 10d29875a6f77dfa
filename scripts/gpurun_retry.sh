#!/bin/bash
# Runs one gpurun call; when the service reports that nothing ran (status
# "transient": no box free, box lost while being prepared, back-off), waits and
# asks again, at most 10 times.  A call that ran is never repeated, whatever
# its exit status.
# usage: scripts/gpurun_retry.sh TIMEOUT_S 'command'
T=$1; shift
for i in $(seq 1 10); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
  echo "[retry] nothing ran (status=$st rc=$rc), waiting" >&2
  sleep 100
done
exit $rc
