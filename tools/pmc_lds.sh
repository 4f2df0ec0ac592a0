# LDS counters of the matrix-free probe for each variant library (VARS), one
# rocprofv3 --pmc pass per variant: bank-conflict cycles against all LDS cycles.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmclds
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in ${VARS}; do
  rm -rf /tmp/pmc
  VAR=$v timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES --kernel-trace --kernel-include-regex "k_mf_pencil" --output-format csv -d /tmp/pmc -o pmc -- python3 $GRAFT_REPO_ROOT/tools/mf_probe.py > $OUT/$v.log 2>&1 || exit $?
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/$v.csv \;
done
