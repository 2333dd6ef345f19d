#!/bin/bash
# rocprofv3 kernel trace + counter passes (one pass per group, each its own run) over any python command, filtered
# to the kernels matching a regex; table via tools/pmc_table.py (dev tool, GPU box).
#   bash tools/pmc_cmd.sh <tag> <kernel-regex> tools/wgrad_bench.py pmc
set -e
TAG=$1; RX=$2; shift 2
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/pmc_$TAG
mkdir -p $D
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $D/trace -o out --output-format csv -- python3 $R/"$@" > $D/log0.txt 2>&1
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_LDS_IDX_ACTIVE" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$RX" -d $D/p$i -o out --output-format csv -- python3 $R/"$@" > $D/log$i.txt 2>&1
done
python3 $R/tools/pmc_table.py $D > $D/table.txt
