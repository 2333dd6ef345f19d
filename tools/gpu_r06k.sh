# tail-kernel LDS change check (dev, GPU box): tail bit-identity + batch-invariance tests, a training trace, the bench
set -e
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-k1}
mkdir -p $D
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_gemm_pp.py tests/test_gpu_dgrad_blaslt.py "tests/test_gpu_fullsize.py::test_c2_batch_equals_single_images" > $D/test.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-infer --no-breakdown > $D/bench_traced.json 2> $D/bench_traced.err
cd $GRAFT_REPO_ROOT && timeout -k 10 600 python -u bench.py --no-cpu-baseline > $D/bench.json 2> $D/bench.err
