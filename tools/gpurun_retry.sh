#!/bin/bash
# Local helper (runs here, not on the GPU box): submit one gpurun call and
# resubmit it only while the pool reports no free box / slot (status
# "transient": nothing ran, nothing charged).  Any other outcome ends it.
#   tools/gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; TO=$2; CMD=$3
for a in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout $TO -- "$CMD" > $LOG 2>&1
  if grep -q "status=transient" $LOG; then echo "[retry $a: no box]" >> $LOG.tries; sleep 150; continue; fi
  break
done
echo done >> $LOG
