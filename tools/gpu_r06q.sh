set -e
mkdir -p gpurun_out/q3
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_gemm_q.py > gpurun_out/q3/test.log 2>&1 || [ $? -eq 1 ]
CFGS=5,6 timeout -k 10 200 python -u tools/gemm_plain.py 8192 > gpurun_out/q3/plain.log 2>&1
AB_ROUNDS=5 timeout -k 10 300 python -u tools/lib_ab.py lin s3od_amd/libs3od_hip.so s3od_amd/libs3od_hip.so@S3OD_GEMM_CFG=6 > gpurun_out/q3/lin.log 2>&1
