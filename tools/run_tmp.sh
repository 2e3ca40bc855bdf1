# temporary experiment driver (GPU box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r03m
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-runs 0 --json-out gpurun_out/${T}_bench.json > gpurun_out/${T}_bench.log 2>&1 || exit $?
NEMO_LIB=var/b256/libnemohip.so timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-runs 0 --json-out gpurun_out/${T}_b256_bench.json > gpurun_out/${T}_b256_bench.log 2>&1 || exit $?
