#!/bin/bash
# round-5 batch: parity (diff, deep tier, C5 digest), diff kernel traces, k_chains_glob phases, the C5 lines
# (resident batch with its CPU baseline, and the configured 1k runs)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r05k}
timeout -k 10 700 python -u -m pytest -x -v --timeout 580 --timeout-method thread tests/test_gpu_diff.py tests/test_gpu_c5_shape.py "tests/test_gpu_parity.py::test_chains_glob_tier" > gpurun_out/${T}_test.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_test.log; [ $rc -le 1 ] || exit $rc
bash tools/prof_diff.sh ${T}_dp || exit 1
bash tools/gpu_glob_phases.sh ${T} 320 || exit 1
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --e2e-runs 0 > gpurun_out/${T}_c5_bench.json 2> gpurun_out/${T}_c5_bench.err || exit 1
timeout -k 10 500 python -u bench.py --config c5 --runs-total 1000 --steps 2 --warmup 1 --e2e-runs 0 > gpurun_out/${T}_c5_1000.json 2> gpurun_out/${T}_c5_1000.err
echo rc=$?
