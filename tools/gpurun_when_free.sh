#!/bin/bash
# Re-submit a gpurun call ONLY while the pool reports no free box / slot (exit 3: nothing ran, nothing
# charged); any other outcome (success, failure, refusal) ends the loop.  Usage: LOG CMD
LOG=$1; shift
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout 1500 -- "$@" > $LOG 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" $LOG; then echo "rc=$rc attempt=$i" >> $LOG; exit $rc; fi
  sleep 150
done
echo "gave up" >> $LOG
