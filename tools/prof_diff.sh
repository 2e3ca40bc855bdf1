#!/bin/bash
# rocprofv3 kernel traces of tools/diff_probe.py (the diff kernels alone), C3 and C5 shapes (run under gpurun)
set -o pipefail
tag=${1:-dp}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in c3 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_$cfg -o kt --output-format csv -- \
    python3 tools/diff_probe.py --config $cfg ${NEMO_PROBE_ARGS} > gpurun_out/${tag}_$cfg.log 2>&1 || exit $?
done
echo ok
