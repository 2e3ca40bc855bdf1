#!/bin/bash
# k_chains_glob per-phase HBM bytes and durations at the C5 shape (stamps build; tools/glob_phases.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/glob_${1:-run}
RUNS=${2:-320}
mkdir -p $OUT
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o kt --output-format csv -- python3 tools/glob_phases.py $RUNS > $OUT/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o f --output-format csv -- python3 tools/glob_phases.py $RUNS > $OUT/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o w --output-format csv -- python3 tools/glob_phases.py $RUNS > $OUT/pmc_write.log 2>&1 && \
python3 tools/glob_phases_sum.py $OUT > $OUT/summary.md 2>&1
echo rc=$?
