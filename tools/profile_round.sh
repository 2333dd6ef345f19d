#!/bin/bash
# Collect the round's rocprofv3 evidence on the GPU box (run from the repo root via gpurun):
#   1. kernel-trace + stats of a short training bench  -> profiles/<tag>_kernel_stats.csv
#   2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) restricted to the roofline kernel
# usage: bash tools/profile_round.sh <tag> [kernel-regex]
set -e
TAG=${1:-r01}
KRE=${2:-attn_fwd_kernel}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer > $OUT/bench_trace.json
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $C --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc_$C -o run -- \
    python $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-infer > $OUT/bench_$C.json
done
ls -R $OUT | head -30
