# round 4: structured-column S (level-major rows, no column indices) and the
# matrix powers: parity files, driver tests, inner-solve A/B under rocprofv3,
# matrix-free pencil variants
set -o pipefail
OUT=gpurun_out/r04i
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_parity_gpu.py tests/test_multi_rank.py::test_group_matrix_powers_bitwise \
  tests/test_cube.py::test_cube_repeated_operator_form_assembly \
  tests/test_driver.py > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "PASSED|FAILED|Error" $OUT/tests.log | head -80; exit 1; }
grep -E "FAILED|passed|failed|matrix powers" $OUT/tests.log | tail -12
for S in 0 1; do
  DCP_S_STRUCT=$S R=5 REPS=3 GS=sstep VAR=none timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_s$S -o inner -- python3 -u tools/inner_probe.py > $OUT/inner_s$S.json 2> $OUT/inner_s$S.err || { echo "inner probe $S failed"; tail -5 $OUT/inner_s$S.err; exit 1; }
  cat $OUT/inner_s$S.json
  f=$(find $OUT/prof_s$S -name "*kernel_stats.csv" | head -1)
  cp "$f" $OUT/inner_s${S}_kernel_stats.csv
  grep -E "k_sell_spmv|k_sstep_block" $OUT/inner_s${S}_kernel_stats.csv | cut -d, -f1-4 | cut -c1-200
done
timeout -k 10 300 python3 -u tools/mf_probe.py > $OUT/mf_variants.json 2> $OUT/mf_variants.err || { echo "mf probe failed"; tail -5 $OUT/mf_variants.err; exit 1; }
cat $OUT/mf_variants.json
echo ALLOK
