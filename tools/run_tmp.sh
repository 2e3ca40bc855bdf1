# temporary experiment driver (GPU box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r03am
timeout -k 10 900 python -u -m pytest tests/test_gpu_deep.py tests/test_gpu_c5_shape.py tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 || exit $?
timeout -k 10 500 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --json-out gpurun_out/${T}_c5_bench.json > gpurun_out/${T}_c5_bench.log 2>&1 || exit $?
timeout -k 10 600 python tools/stamps_glob.py 320 1000000 2000 dense > gpurun_out/${T}_stamps_glob320.txt 2>&1 || exit $?
