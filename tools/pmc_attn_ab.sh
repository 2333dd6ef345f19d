#!/bin/bash
# SQ counter passes over tools/attn_ab.py (both settings of a knob in one process: the kernels of both appear), GPU box.
# usage: bash tools/pmc_attn_ab.sh <tag> <knob> <val1> <val2>
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-pmc_attn_ab}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for G in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  AB_ROUNDS=1 AB_SMALL=1 timeout -k 10 240 rocprofv3 --pmc $G --kernel-include-regex "attn_bwd" --output-format csv -d $OUT/p$i -o run -- \
    python3 $GRAFT_REPO_ROOT/tools/attn_ab.py $2 $3 $4 > $OUT/p$i.log 2>&1 || exit 1
done
python3 $GRAFT_REPO_ROOT/tools/pmc_table.py $OUT > $OUT/table.txt
cat $OUT/table.txt
