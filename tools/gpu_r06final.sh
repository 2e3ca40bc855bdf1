#!/bin/bash
# round-6 final measurements (run under gpurun, one part per call):
#   a: the whole GPU suite, smoke, tools/prof_bench.sh of the driver's C3 line
#   b: tools/prof_bench.sh of the per-run diff line and of the C5 resident line
#   c: the C5 1k-run line (with its CPU baseline), diff kernel traces
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
case "$1" in
a)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r06final_gputest.log 2>&1
  rc=$?; tail -3 gpurun_out/r06final_gputest.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06final_smoke.log 2>&1 || exit 1
  tail -1 gpurun_out/r06final_smoke.log
  bash tools/prof_bench.sh r06 || exit 1 ;;
b)
  bash tools/prof_bench.sh r06_perrun --diff-mode per_run || exit 1
  bash tools/prof_bench.sh r06_c5 --config c5 --steps 2 --warmup 1 --e2e-runs 0 || exit 1 ;;
c)
  timeout -k 10 600 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 > gpurun_out/r06final_c5_1000.json 2> gpurun_out/r06final_c5_1000.err || exit 1
  bash tools/prof_diff.sh r06final_dp || exit 1 ;;
esac
echo part $1 done
case "$1" in
z)  # after the last library change: the whole GPU suite, smoke, the driver's C3 line
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r06z_gputest.log 2>&1
  rc=$?; tail -3 gpurun_out/r06z_gputest.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06z_smoke.log 2>&1 || exit 1
  tail -1 gpurun_out/r06z_smoke.log
  timeout -k 10 400 python -u bench.py > gpurun_out/r06z_bench.json 2> gpurun_out/r06z_bench.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r06z_bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['e2e']['runs_per_s'] if d.get('e2e') else None)" ;;
esac
