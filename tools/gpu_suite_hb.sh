# The GPU test suite with a heartbeat file under gpurun_out/ (a test that
# runs silently for minutes is not taken for a hang), then the smoke.
# usage: TAG=r06v bash tools/gpu_suite_hb.sh [pytest args...]
set -u
TAG=${TAG:-gpu}
mkdir -p gpurun_out
( while true; do date >> gpurun_out/${TAG}_gputests.hb; sleep 50; done ) &
HB=$!
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread "$@" > gpurun_out/${TAG}_gputests.log 2>&1
RC=$?
kill $HB
echo "gpu tests rc=$RC"
[ $RC -eq 0 ] || exit $RC
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
echo "smoke rc=$?"
