#!/bin/bash
# PMC passes over one probe of a stand-alone probe binary (counters only with
# --kernel-trace; each pass its own run under a hard time limit).
# usage: scripts/pmc_probe.sh OUTDIR KERNEL_REGEX -- <probe command...>
set -u -o pipefail
OUT=$1; shift
RX=$1; shift; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $set --kernel-trace --kernel-include-regex "$RX" --output-format csv -d "$OUT/p$i" -o pmc -- "$@" > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.log"; exit $rc; fi
done
