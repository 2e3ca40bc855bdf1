#!/bin/bash
# A/B of C3 variants (var/NAME/libnemohip.so) against the in-tree library: bench.py's C3 line, step and kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-c3var}; shift
for v in base "$@"; do
  if [ $v = base ]; then lib=""; else lib="NEMO_LIB=var/$v/libnemohip.so"; fi
  env $lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --e2e-runs 0 --no-cpu-baseline --diff-reps 0 > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || exit 1
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/${T}_$v.json').read().strip().splitlines()[-1]);print('$v',d['value'],d['ms_per_step'],{k:round(x['ms_total']/x['launches'],3) for k,x in d['kernels'].items() if x['ms_total']/x['launches']>0.1})"
done
