#!/bin/bash
# One step of a gpurun call: `tools/gpu_job.sh TAG SECONDS cmd args...` runs
# cmd under `timeout -k 10 SECONDS` with stdout+stderr in gpurun_out/TAG.log,
# a heartbeat line per minute in gpurun_out/TAG.hb (long steps stay visibly
# alive), and prints the log's tail on failure. Chain steps with &&.
set -o pipefail
TAG=$1; LIMIT=$2; shift 2
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
( while sleep 50; do date +%T >> gpurun_out/$TAG.hb; done ) &
HB=$!
timeout -k 10 "$LIMIT" "$@" > gpurun_out/$TAG.log 2>&1
rc=$?
kill $HB 2>/dev/null
if [ $rc -ne 0 ]; then
  echo "step $TAG failed rc=$rc"; tail -30 gpurun_out/$TAG.log; exit $rc
fi
echo "step $TAG ok"; tail -3 gpurun_out/$TAG.log
