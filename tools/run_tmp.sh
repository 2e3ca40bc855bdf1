# temporary experiment driver (GPU box)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r03ac
for v in main sb8 sb2 td2 td8; do
  if [ $v = main ]; then L=; else L=var/$v/libnemohip.so; fi
  NEMO_LIB=$L timeout -k 10 500 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --json-out gpurun_out/${T}_${v}_c5_bench.json > gpurun_out/${T}_${v}_c5_bench.log 2>&1 || exit $?
done
