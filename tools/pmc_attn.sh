#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per launch of the attention kernels (separate PMC passes) over tools/kprobe.py attn
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_attn
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "attn" --output-format csv -d $OUT/$C -o run -- \
    python $GRAFT_REPO_ROOT/tools/kprobe.py attn > $OUT/$C.log 2>&1
done
