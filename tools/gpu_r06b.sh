set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_attention_fullsize.py tests/test_gpu_conv_halo.py tests/test_gpu_knob_once.py tests/test_gpu_colsum.py > gpurun_out/r06b/t1.log 2>&1 || { tail -30 gpurun_out/r06b/t1.log; exit 1; }
tail -3 gpurun_out/r06b/t1.log
MIOPEN_FIND_MODE=FAST MIOPEN_USER_DB_PATH=/tmp/mu1 MIOPEN_CUSTOM_CACHE_DIR=/tmp/mc1 timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 880 --timeout-method thread "tests/test_gpu_fullsize.py::test_c5_one_image_strict_vs_oracle" > gpurun_out/r06b/c5_fast.log 2>&1 || { tail -20 gpurun_out/r06b/c5_fast.log; exit 1; }
grep -E "phases|passed|failed" gpurun_out/r06b/c5_fast.log
MIOPEN_USER_DB_PATH=/tmp/mu2 MIOPEN_CUSTOM_CACHE_DIR=/tmp/mc2 timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 880 --timeout-method thread "tests/test_gpu_fullsize.py::test_c5_one_image_strict_vs_oracle" > gpurun_out/r06b/c5_default.log 2>&1 || { tail -20 gpurun_out/r06b/c5_default.log; exit 1; }
grep -E "phases|passed|failed" gpurun_out/r06b/c5_default.log
