#!/bin/bash
# A/B of library variants (var/NAME/libnemohip.so) on the per-run diff line (roofline_diff), twice each
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=$1; shift
for rep in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then lib=""; else lib="NEMO_LIB=var/$v/libnemohip.so"; fi
    env $lib timeout -k 10 300 python -u bench.py --diff-mode per_run --no-cpu-baseline --e2e-runs 0 --steps 3 > gpurun_out/${T}_${rep}_$v.json 2> gpurun_out/${T}_${rep}_$v.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${rep}_$v.json').read().strip().splitlines()[-1]);r=d['roofline_diff'];print('$v',r['avg_launch_ms'],r['frac'],d['ms_per_step'])"
  done
done
