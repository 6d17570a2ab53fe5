#!/bin/bash
# gpurun client retry on infrastructure errors (rc 3: no box / box not prepared; nothing ran)
out=$1; shift
for i in 1 2 3 4 5; do
  /usr/local/graft/bin/gpurun "$@" > "$out" 2>&1
  rc=$?
  echo "rc=$rc" >> "$out"
  [ $rc -ne 3 ] && exit $rc
  sleep 60
done
exit 3
