#!/bin/bash
# queue a gpurun call: retries only while gpurun answers 3 (no box or slot free: nothing ran, nothing
# charged); any other exit (including a failed command) ends it.  usage: tools/gpuq.sh TIMEOUT 'cmd'
t=$1; shift
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $t -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
exit 3
