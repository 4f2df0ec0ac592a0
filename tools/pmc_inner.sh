# HBM traffic of the inner Schur GMRES kernels at r=5 (tools/inner_probe.py,
# GS=classical2 by default, GS=sstep for the s-step blocks): one rocprofv3
# --pmc pass per counter, summarised by tools/pmc_summary.py into
# gpurun_out/<TAG>_pmc_inner/summary.json. KREGEX: the kernels counted.
set -u
TAG=${TAG:-r03}
KREGEX=${KREGEX:-k_sell_spmv|k_cgs2_chain|k_dcgs2}
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG}_pmc_inner
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc
  R=5 REPS=2 GS=${GS:-classical2} timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "$KREGEX" --output-format csv -d /tmp/pmc -o pmc -- python3 $GRAFT_REPO_ROOT/tools/inner_probe.py > $OUT/$ctr.log 2>&1 || exit $?
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/$ctr.csv \;
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT "rocprofv3 --pmc <CTR> --kernel-trace --kernel-include-regex '$KREGEX' -- python3 tools/inner_probe.py (R=5 REPS=2 GS=${GS:-classical2})" $OUT/summary.json
rm -f $OUT/*.csv
