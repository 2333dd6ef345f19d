#!/bin/bash
# GEMM tile-config sweep of the ViT linears with their real epilogues (dev tool, GPU box)
OUT=gpurun_out/${1:-sweep}; mkdir -p $OUT
for c in -1 0 1 3 4; do
  S3OD_GEMM_CFG=$c timeout -k 10 200 python -u tools/lin_sweep.py >> $OUT/lin_sweep.txt 2>&1 || exit $?
done
