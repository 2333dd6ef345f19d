#!/bin/bash
# Stall / occupancy / instruction-mix counters of the attention-backward kernels at the training shape (bs 16, N 4101),
# one rocprofv3 pass per counter group (each within the per-pass slot limits), GPU box.  Table via tools/pmc_table.py.
#   bash tools/pmc_attn_stall.sh <tag> [kernel-regex] [probe args...]
# Derived in the table: occupancy = SQ_WAVE_CYCLES*4 / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs), wait fractions of SQ_WAVE_CYCLES.
set -e
TAG=$1; RX=${2:-attn_bwd}; shift 2 || true
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/pmc_$TAG
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
PROBE=${PROBE:-tools/kprobe.py attn}
timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $D/trace -o out --output-format csv -- python3 $R/$PROBE > $D/log0.txt 2>&1
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE" \
         "SQ_VALU_MFMA_COEXEC_CYCLES SQ_INST_LEVEL_LDS SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex "$RX" -d $D/p$i -o out --output-format csv -- python3 $R/$PROBE > $D/log$i.txt 2>&1
done
python3 $R/tools/pmc_table.py $D > $D/table.txt
cat $D/table.txt
