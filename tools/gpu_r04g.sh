# round 4: matrix-powers bitwise tests, driver tests, the whole GPU suite,
# smoke, bench r=5, then the matrix-free pencil variants (tools/mf_probe.py)
set -o pipefail
OUT=gpurun_out/r04g
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_multi_rank.py::test_group_matrix_powers_bitwise \
  tests/test_parity_gpu.py::test_repeated_operator_form_assembly_matches_oracle \
  tests/test_cube.py::test_cube_repeated_operator_form_assembly \
  tests/test_driver.py > $OUT/new_tests.log 2>&1 || { echo "new tests failed"; grep -E "PASSED|FAILED|Error" $OUT/new_tests.log | head -60; exit 1; }
grep -E "PASSED|FAILED|matrix powers|scatter info" $OUT/new_tests.log | tail -40
timeout -k 10 300 python3 -u tools/mf_probe.py > $OUT/mf_variants.json 2> $OUT/mf_variants.err || { echo "mf probe failed"; tail -5 $OUT/mf_variants.err; exit 1; }
cat $OUT/mf_variants.json
echo ALLOK
