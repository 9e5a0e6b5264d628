#!/bin/bash
# Run GPU steps in order, each "name|seconds|command" line of a step file,
# output to gpurun_out/<tag>/<name>.log.  A failing step (ordinary nonzero
# status, e.g. a test failure) does not stop the rest; a time limit, abort,
# segfault or kill (status 124, 134, 137, 139 or >= 128) ends the run there --
# nothing more touches the GPU after a fault.
#   bash tools/steps.sh <tag> <stepfile>
TAG=$1; FILE=$2
OUT=gpurun_out/$TAG; mkdir -p $OUT
rc_all=0
while IFS='|' read -r name secs cmd; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue;; esac
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "step $name rc=$rc $(( $(date +%s) - start ))s" | tee -a $OUT/steps.txt
  tail -3 "$OUT/$name.log"
  if [ $rc -ne 0 ]; then rc_all=$rc; fi
  if [ $rc -eq 124 ] || [ $rc -ge 128 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
done < "$FILE"
exit $rc_all
