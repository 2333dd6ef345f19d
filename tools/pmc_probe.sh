#!/bin/bash
# Per-kernel SQ counter passes over tools/kprobe.py (one counter group per pass).
# usage: bash tools/pmc_probe.sh <outdir-name> [which]
set -e
NAME=${1:-probe}
WHICH=${2:-all}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
         "SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU" \
         "SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o run -- \
    python $GRAFT_REPO_ROOT/tools/kprobe.py $WHICH > $OUT/p$i.log 2>&1
done
echo done
