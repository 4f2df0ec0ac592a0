# HBM traffic of the matrix-free Stokes apply (tools/mf_probe.py, r=5): one
# rocprofv3 --pmc pass per counter (FETCH_SIZE, WRITE_SIZE), summarised with
# tools/pmc_summary.py into gpurun_out/pmcmf2/summary.json.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcmf2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc
  R=5 timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "k_mf_pencil|k_mf_gather" --output-format csv -d /tmp/pmc -o pmc -- python3 $GRAFT_REPO_ROOT/tools/mf_probe.py > $OUT/$ctr.log 2>&1 || exit $?
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/$ctr.csv \;
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT "rocprofv3 --pmc <CTR> --kernel-trace --kernel-include-regex 'k_mf_pencil|k_mf_gather' -- python3 tools/mf_probe.py (R=5)" $OUT/summary.json
rm -f $OUT/*.csv
