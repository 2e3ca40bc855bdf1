# temporary experiment driver (GPU box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r03s
for v in main odd main2 odd2; do
  case $v in main*) L=;; *) L=var/${v%2}/libnemohip.so;; esac
  NEMO_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-runs 0 --json-out gpurun_out/${T}_${v}_bench.json > gpurun_out/${T}_${v}_bench.log 2>&1 || exit $?
done
