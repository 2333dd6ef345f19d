# GEMM default change check + a training kernel trace (dev, GPU box)
set -e
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-t1}
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_gemm_pp.py tests/test_gpu_train.py tests/test_gpu_forward.py tests/test_gpu_parity_holes.py > $D/test.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace_train -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-breakdown > $D/bench_train.json 2> $D/bench_train.err
