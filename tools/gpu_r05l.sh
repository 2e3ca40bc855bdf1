#!/bin/bash
# round-5 batch: the whole GPU suite, smoke, the C3 tunable A/B, the C5 1k-run line
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r05l}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1
rc=$?; tail -3 gpurun_out/${T}_gputest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
tail -2 gpurun_out/${T}_smoke.log
bash tools/gpu_c3var.sh ${T}_c3v pr64 pr160 chk4 chk2 || exit 1
timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 > gpurun_out/${T}_c5_1000.json 2> gpurun_out/${T}_c5_1000.err
echo rc=$?
