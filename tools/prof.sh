#!/bin/bash
# rocprofv3 kernel-trace stats + SQ counter passes for the pipeline (GPU box).
set -e
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/prof_${1:-run}
shift || true
mkdir -p $OUT
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o kt --output-format csv -- python3 tools/prof_pipeline.py 2000 3 "$@" > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU -d $OUT/pmc1 -o p1 --output-format csv -- python3 tools/prof_pipeline.py 2000 1 "$@" > $OUT/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc2 -o p2 --output-format csv -- python3 tools/prof_pipeline.py 2000 1 "$@" > $OUT/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc3 -o p3 --output-format csv -- python3 tools/prof_pipeline.py 2000 1 "$@" > $OUT/pmc3.log 2>&1
echo done
