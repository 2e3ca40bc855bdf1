#!/bin/bash
# round-5 final batch: the whole GPU suite, smoke, the driver's C3 line and the per-run diff line
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r05f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_gputest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/${T}_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
timeout -k 10 400 python -u bench.py --diff-mode per_run --no-cpu-baseline --e2e-runs 0 > gpurun_out/${T}_perrun.json 2> gpurun_out/${T}_perrun.err
echo rc=$?
