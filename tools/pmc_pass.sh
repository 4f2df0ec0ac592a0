# HBM traffic (rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE: one counter per
# pass) of the kernels matching REGEX in one probe run, summarised by
# tools/pmc_summary.py (2*FETCH + WRITE per dispatch, the gfx950 correction)
# into gpurun_out/$TAG/summary.json.  usage: TAG=.. REGEX=.. bash tools/pmc_pass.sh <probe.py>
set -u
PROBE=$1
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "$REGEX" --output-format csv -d /tmp/pmc -o pmc -- python3 $GRAFT_REPO_ROOT/$PROBE > $OUT/$ctr.log 2>&1 || exit $?
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/$ctr.csv \;
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT "rocprofv3 --pmc <CTR> --kernel-trace --kernel-include-regex '$REGEX' -- python3 $PROBE" $OUT/summary.json
rm -f $OUT/*.csv
