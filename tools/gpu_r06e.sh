# epilogue rework measurements (dev, GPU box): GPU tests (all but the full-size ones), block timeline, ViT linears
# A/B vs old_lib, plain GEMM K fit
set -e
D=gpurun_out/${TAG:-e1}
mkdir -p $D
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread -k "not fullsize" tests > $D/test.log 2>&1
timeout -k 10 200 python -u tools/pp_timeline.py > $D/tl.log 2>&1
AB_ROUNDS=5 timeout -k 10 300 python -u tools/lib_ab.py lin old_lib/libs3od_hip.so s3od_amd/libs3od_hip.so > $D/lin.log 2>&1
CFGS=5 timeout -k 10 300 python -u tools/gemm_plain.py kfit > $D/kfit.log 2>&1
