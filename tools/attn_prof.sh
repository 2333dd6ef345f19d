#!/bin/bash
# rocprofv3 kernel stats + two SQ counter passes over tools/kprobe.py attn (GPU box)
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-attn_prof}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python $GRAFT_REPO_ROOT/tools/kprobe.py attn > $OUT/stats.log 2>&1 || exit 1
i=0
for G in "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $G --output-format csv -d $OUT/p$i -o run -- python $GRAFT_REPO_ROOT/tools/kprobe.py attn > $OUT/p$i.log 2>&1 || exit 1
done
python $GRAFT_REPO_ROOT/tools/pmc_table.py $OUT > $OUT/table.txt
find $OUT/stats -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-5 | head -12
