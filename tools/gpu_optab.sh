#!/bin/bash
# A/B of library options on the driver's C3 line: bench.py with each --set list (quoted), alternating, twice
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=$1; shift
for rep in 1 2; do
  i=0
  for opts in "" "$@"; do
    args=""; for o in $opts; do args="$args --set $o"; done
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --e2e-runs 0 --no-cpu-baseline --diff-reps 0 $args > gpurun_out/${T}_${rep}_$i.json 2> gpurun_out/${T}_${rep}_$i.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/${T}_${rep}_$i.json').read().strip().splitlines()[-1]);print('[$opts]',d['value'],d['ms_per_step'],{k:round(x['ms_total']/x['launches'],3) for k,x in d['kernels'].items() if x['ms_total']/x['launches']>0.1})"
    i=$((i+1))
  done
done
