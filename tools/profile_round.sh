#!/bin/bash
# Collect the round's rocprofv3 evidence on the GPU box (run from the repo root via gpurun):
#   1. kernel trace + stats of a short training bench (configs[2])          -> trace_train
#      the same with the whole backward on one stream (--single-stream)    -> trace_train_ss
#   2. separate PMC passes FETCH_SIZE / WRITE_SIZE on the roofline kernel   -> pmc_train_<C>
#   3. kernel trace + stats of the 2048^2 bs=4 inference bench (configs[4]) -> trace_c5
#   4. separate PMC passes FETCH_SIZE / WRITE_SIZE over every C5 kernel     -> pmc_c5_<C>
# Each step has its own time limit; steps are chained with && (nothing runs after a failure).
# usage: bash tools/profile_round.sh <tag> [roofline-kernel-regex]
TAG=${1:-r02}
KRE=${2:-attn_(bwd|delta)}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B=$GRAFT_REPO_ROOT/bench.py
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train -o run -- \
  python3 $B --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-breakdown > $OUT/bench_train.json 2> $OUT/bench_train.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_train_ss -o run -- \
  python3 $B --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-breakdown --single-stream > $OUT/bench_train_ss.json 2> $OUT/bench_train_ss.err && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc_train_FETCH_SIZE -o run -- \
  python3 $B --steps 1 --warmup 1 --no-cpu-baseline --no-infer --no-breakdown > /dev/null 2> $OUT/pmc_train_f.err && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" --output-format csv -d $OUT/pmc_train_WRITE_SIZE -o run -- \
  python3 $B --steps 1 --warmup 1 --no-cpu-baseline --no-infer --no-breakdown > /dev/null 2> $OUT/pmc_train_w.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c5 -o run -- \
  python3 $B --mode infer --batch 4 --size 2048 --steps 3 --warmup 1 --no-cpu-baseline --no-breakdown > $OUT/bench_c5.json 2> $OUT/bench_c5.err && \
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_c5_FETCH_SIZE -o run -- \
  python3 $B --mode infer --batch 4 --size 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-breakdown > /dev/null 2> $OUT/pmc_c5_f.err && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_c5_WRITE_SIZE -o run -- \
  python3 $B --mode infer --batch 4 --size 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-breakdown > /dev/null 2> $OUT/pmc_c5_w.err
rc=$?
find $OUT -name "*.csv" | head -30
exit $rc
