#!/bin/bash
# wait for a free GPU box: re-issue the same gpurun call only while it reports "no box / slot free" (exit 3,
# nothing ran, nothing charged); any other outcome is returned as is
for i in $(seq 1 ${TRIES:-20}); do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep ${WAIT:-90}
done
exit 3
