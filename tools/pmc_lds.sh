#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc_lds
mkdir -p $OUT
cd $R
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAVES -d $OUT/p1 -o p1 --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --e2e-runs 0 > $OUT/p1.log 2>&1
echo done
