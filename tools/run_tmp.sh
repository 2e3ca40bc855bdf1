# temporary experiment driver (GPU box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r03ak
NEMO_LIB=var/g512/libnemohip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.log 2>&1 || exit $?
for v in base g160 g256 g512; do
  NEMO_LIB=var/$v/libnemohip.so timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-runs 0 --json-out gpurun_out/${T}_${v}_bench.json > gpurun_out/${T}_${v}_bench.log 2>&1 || exit $?
done
