#!/bin/bash
# quick GPU regression: train / forward / parity-hole / checkpoint / dinol tests, then the bench without CPU baseline
OUT=gpurun_out/${1:-quick}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_forward.py tests/test_gpu_parity_holes.py tests/test_gpu_checkpoint.py tests/test_gpu_dinol.py tests/test_gpu_lightning.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -3 $OUT/gpu_tests.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; echo "bench rc=$?"
