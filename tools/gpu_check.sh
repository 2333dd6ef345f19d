#!/bin/bash
# One GPU-box pass (run through gpurun from the repo root): the -m gpu suite, then (only if pytest
# ended normally: rc 0 = green, 1 = failures; never after a crash / timeout) the default bench.
# usage: bash tools/gpu_check.sh <tag> [pytest selection...]
TAG=${1:-chk}
shift
SEL=${@:-tests}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
tail -5 $OUT/gpu_tests.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 720 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
  brc=$?
  echo "bench rc=$brc"
  tail -c 3000 $OUT/bench.json
  exit $brc
fi
exit $rc
