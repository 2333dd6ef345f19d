#!/bin/bash
# A/B of the bf16 attention-backward launch knobs (GPU box): one process per variant, then a rocprofv3
# kernel-stats pass of the default to split the time between the dK/dV and dQ passes.
OUT=gpurun_out/${1:-attn_ab}; mkdir -p $OUT
for v in "4 4 0 1" "4 4 0 0" "4 4 0 1" "4 4 0 0"; do
  set -- $v
  S3OD_ATTN_WK=$1 S3OD_ATTN_WQ=$2 S3OD_ATTN_PRIO=$3 S3OD_ATTN_IL=$4 timeout -k 10 200 python tools/attn_sweep.py $OUT/x.pt >> $OUT/sweep.txt 2>&1 || exit 1
done
rm -f $OUT/x.pt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python $GRAFT_REPO_ROOT/tools/attn_sweep.py $GRAFT_REPO_ROOT/$OUT/x.pt > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1
rm -f $GRAFT_REPO_ROOT/$OUT/x.pt
cat $GRAFT_REPO_ROOT/$OUT/sweep.txt | grep -v amdgpu.ids
find $GRAFT_REPO_ROOT/$OUT/prof -name "*kernel_stats.csv" -exec head -8 {} \;
