# GEMM tile-order / fixed-cost measurements (dev, GPU box): plain 8192^3 + ViT shapes per S3OD_GEMM_GROUP, the
# time-vs-K fit, the ViT linears A/B (row-major vs grouped tile order)
set -e
D=gpurun_out/${TAG:-g1}
mkdir -p $D
for G in 0 4 8; do
  S3OD_GEMM_GROUP=$G CFGS=5,6 timeout -k 10 200 python -u tools/gemm_plain.py 8192 > $D/plain_g$G.log 2>&1
done
CFGS=5 timeout -k 10 300 python -u tools/gemm_plain.py kfit > $D/kfit.log 2>&1
L=s3od_amd/libs3od_hip.so
AB_ROUNDS=5 timeout -k 10 300 python -u tools/lib_ab.py lin $L $L@S3OD_GEMM_GROUP=4 $L@S3OD_GEMM_GROUP=8 > $D/lin.log 2>&1
