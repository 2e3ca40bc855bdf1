#!/bin/bash
# round-6 GPU steps (run under gpurun, one part per call); every GPU step has its own time limit
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
tag=${2:-r06}
case "$1" in
new)  # the round's new tests first, then the whole suite
  timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_batched.py \
    tests/test_gpu_diff.py tests/test_gpu_parity.py::test_stage_and_diff_streams > gpurun_out/${tag}_new.log 2>&1
  rc=$?; tail -5 gpurun_out/${tag}_new.log; [ $rc -eq 0 ] || exit $rc ;;
suite)
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_suite.log 2>&1
  rc=$?; tail -3 gpurun_out/${tag}_suite.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || exit 1
  tail -1 gpurun_out/${tag}_smoke.log ;;
bench)
  timeout -k 10 400 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${tag}_bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['kernel'],d['roofline']['frac'])" ;;
esac
echo part $1 done
