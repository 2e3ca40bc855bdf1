#!/bin/bash
# GPU-box steps of a round-4 measurement (run through gpurun from the repo root):
#   tests (optional) -> bench C3 (+ per_run diff leg) -> bench C5 (+ per_run diff leg)
# Each GPU step has its own time limit; a failing step ends the script.
set -o pipefail
tag=${1:-r04}
mode=${2:-all}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "$mode" = all ] || [ "$mode" = tests ]; then
  timeout -k 10 900 python -u -m pytest ${NEMO_TESTS:-tests} -m gpu -x -v --timeout 900 --timeout-method thread \
    ${NEMO_K:+-k "$NEMO_K"} ${NEMO_PYTEST_ARGS} > gpurun_out/${tag}_gputest.log 2>&1 || exit $?
fi
if [ "$mode" = all ] || [ "$mode" = bench ] || [ "$mode" = benches ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline --e2e-runs 0 ${NEMO_BENCH_ARGS} --json-out gpurun_out/${tag}_bench.json > gpurun_out/${tag}_bench.log 2>&1 || exit $?
fi
if [ "$mode" = all ] || [ "$mode" = c5 ] || [ "$mode" = benches ]; then
  timeout -k 10 500 python bench.py --config c5 --steps ${C5_STEPS:-2} --warmup 1 --no-cpu-baseline --diff-reps ${C5_DIFF_REPS:-2} ${NEMO_C5_ARGS} \
    --json-out gpurun_out/${tag}_c5_bench.json > gpurun_out/${tag}_c5_bench.log 2>&1 || exit $?
fi
echo ok
