#!/bin/bash
# GPU-box steps of a round-3 verification (run through gpurun from the repo root):
#   tests  -> pytest -m gpu (all, or $NEMO_TESTS), then bench C3 -> gpurun_out/<tag>_*
# Each GPU step has its own time limit; a failing step ends the script.
set -o pipefail
tag=${1:-r03}
mode=${2:-all}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
{ cat /sys/fs/cgroup/cpu.max; nproc; python -c "import os; print(len(os.sched_getaffinity(0)))"; } > gpurun_out/${tag}_box_cpu.txt 2>&1
if [ "$mode" = all ] || [ "$mode" = tests ]; then
  timeout -k 10 900 python -u -m pytest ${NEMO_TESTS:-tests} -m gpu -x -v --timeout 900 --timeout-method thread \
    ${NEMO_K:+-k "$NEMO_K"} ${NEMO_PYTEST_ARGS} > gpurun_out/${tag}_gputest.log 2>&1 || exit $?
fi
if [ "$mode" = all ] || [ "$mode" = bench ]; then
  timeout -k 10 400 python bench.py ${NEMO_BENCH_ARGS} --json-out gpurun_out/${tag}_bench.json > gpurun_out/${tag}_bench.log 2>&1 || exit $?
fi
if [ "$mode" = all ] || [ "$mode" = c5 ]; then
  timeout -k 10 500 python bench.py --config c5 --steps ${C5_STEPS:-3} --warmup 1 ${NEMO_C5_ARGS} \
    --json-out gpurun_out/${tag}_c5_bench.json > gpurun_out/${tag}_c5_bench.log 2>&1 || exit $?
fi
