#!/bin/bash
# Round profile of bench.py on the GPU box (run under gpurun):
#   1. bench.py as the driver runs it                       -> bench.json
#   2. the same command under rocprofv3 --kernel-trace --stats -> trace/
#   3. separate PMC passes (HBM bytes, SQ occupancy/stalls)   -> pmc_*/
# tools/pmc_summary.py turns the CSVs into profiles/.
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof_${1:-run}
shift || true
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --e2e-runs 0 "$@" > $OUT/trace.log 2>&1
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o f --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --e2e-runs 0 "$@" > $OUT/pmc_fetch.log 2>&1
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o w --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --e2e-runs 0 "$@" > $OUT/pmc_write.log 2>&1
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d $OUT/pmc_sq -o s --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --e2e-runs 0 "$@" > $OUT/pmc_sq.log 2>&1
echo done
