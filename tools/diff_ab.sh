#!/bin/bash
# A/B of the per-run diff call (tools/diff_probe.py, C3) over library variants (var/NAME/libnemohip.so)
cd $GRAFT_REPO_ROOT
for v in base "$@"; do
  if [ $v = base ]; then unset NEMO_LIB; else export NEMO_LIB=$PWD/var/$v/libnemohip.so; fi
  for r in 1 2; do
    timeout -k 10 200 python tools/diff_probe.py --config c3 2>/dev/null | grep -o '"k_diff_ms": [0-9.]*' | sed "s/^/$v /" || exit 1
  done
done
