#!/bin/bash
# Kernel trace of bench.py (no CPU / e2e legs) -> gpurun_out/trace_<tag>/
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/trace_${1:-run}
shift || true
mkdir -p $OUT
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --e2e-runs 0 "$@" > $OUT/trace.log 2>&1
echo done
