# deep-tier check on the GPU box: deep parity tests, then the C5 bench (diagnostic)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_deep.py \
  "tests/test_gpu_parity.py::test_large_graphs_global_paths" "tests/test_gpu_parity.py::test_dense_c5_shape" \
  "tests/test_gpu_parity.py::test_global_tier_block" "tests/test_gpu_parity.py::test_chains_glob_tier" \
  tests/test_gpu_scale.py::test_c5_deep_graphs_default_tiers > gpurun_out/deep_tests_$T.log 2>&1 && \
timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --e2e-runs 0 > gpurun_out/bench_c5_$T.json 2> gpurun_out/bench_c5_$T.err
echo rc=$?
if [ "$2" = "stamps" ]; then
  timeout -k 10 300 python tools/stamps_glob.py 4 1000000 2000 dense > gpurun_out/stamps_glob_$T.txt 2>&1
fi
