# Round-end GPU evidence (dev, GPU box): the whole GPU test suite, smoke(), then the default bench line.
set -e
D=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-final}
mkdir -p $D
timeout -k 10 1500 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests > $D/gpu_tests.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1
timeout -k 10 900 python -u bench.py > $D/bench_full.json 2> $D/bench_full.err
