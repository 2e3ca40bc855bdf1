set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r02c.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_r02c.json 2> gpurun_out/bench_r02c.err && \
timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --e2e-runs 0 > gpurun_out/bench_c5_r02c.json 2> gpurun_out/bench_c5_r02c.err
echo rc=$?
