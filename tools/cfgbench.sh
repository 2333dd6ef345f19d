set -e
for c in 0 1 2; do echo "== cfg $c"; S3OD_GEMM_CFG=$c timeout -k 10 200 python tools/gemm_bench.py; done
