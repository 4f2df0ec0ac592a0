# HBM traffic (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one pass per counter)
# of the operator-form NSE assembly (tools/asm_probe.py: 6 assemblies at r=5)
# and of the temperature assembly (tools/tsep_probe.py, PROBES=0), summarised
# with tools/pmc_summary.py (2 FETCH + WRITE, the gfx950 correction).
set -u
TAG=${TAG:-r06w}
OUT=gpurun_out/${TAG}_pmc
mkdir -p $OUT/asm $OUT/tsep
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc
  timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "k_btk|k_bt_tasks|k_mf_pencil|k_mf_gather|k_nse_rhs_halfwave|k_con_gather|k_cdk" --output-format csv -d /tmp/pmc -o pmc -- python3 tools/asm_probe.py > $OUT/asm_$ctr.log 2>&1 || exit 1
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/asm/$ctr.csv \;
  rm -rf /tmp/pmc
  PROBES=0 REPS=6 timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "k_tsep" --output-format csv -d /tmp/pmc -o pmc -- python3 tools/tsep_probe.py > $OUT/tsep_$ctr.log 2>&1 || exit 1
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/tsep/$ctr.csv \;
done
python3 tools/pmc_summary.py $OUT/asm "rocprofv3 --pmc <CTR> --kernel-trace --kernel-include-regex 'k_btk|k_bt_tasks|k_mf_pencil|k_mf_gather|k_nse_rhs_halfwave|k_con_gather|k_cdk' -- python3 tools/asm_probe.py (R=5)" $OUT/pmc_asm_r5.json || exit 1
python3 tools/pmc_summary.py $OUT/tsep "rocprofv3 --pmc <CTR> --kernel-trace --kernel-include-regex k_tsep -- python3 tools/tsep_probe.py (R=5, PROBES=0, REPS=6)" $OUT/pmc_tsep_r5.json || exit 1
rm -f $OUT/asm/*.csv $OUT/tsep/*.csv
echo done
