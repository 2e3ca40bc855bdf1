# temporary experiment driver (GPU box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r03aj
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_golden.py tests/test_gpu_deep.py tests/test_gpu_c5_shape.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 || exit $?
for v in main main2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-runs 0 --json-out gpurun_out/${T}_${v}_bench.json > gpurun_out/${T}_${v}_bench.log 2>&1 || exit $?
done
timeout -k 10 500 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --json-out gpurun_out/${T}_c5_bench.json > gpurun_out/${T}_c5_bench.log 2>&1 || exit $?
