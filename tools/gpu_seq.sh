#!/bin/bash
# Several gpu_job.sh steps in one gpurun call: `tools/gpu_seq.sh "TAG SECS cmd..." ...`.
# A step that ends with 0 or 1 (pytest: tests ran, some may have failed) lets
# the next one start; anything else (a fault, an abort, a time limit) ends the
# call there.
rc_all=0
for step in "$@"; do
  eval "tools/gpu_job.sh $step"
  rc=$?
  [ $rc -ne 0 ] && rc_all=$rc
  if [ $rc -gt 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
exit $rc_all
