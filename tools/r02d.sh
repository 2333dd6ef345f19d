set -o pipefail
OUT=gpurun_out/r02d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dinol.py -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1; rc=$?
tail -3 $OUT/gpu_tests.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/step_profile.py --mode train > $OUT/step_train.txt 2>&1 && \
timeout -k 10 300 python -u tools/step_profile.py --mode infer --batch 8 > $OUT/step_infer.txt 2>&1 && \
timeout -k 10 300 python -u tools/step_profile.py --mode infer --batch 4 --size 2048 > $OUT/step_infer2048.txt 2>&1
echo "profile rc=$?"
