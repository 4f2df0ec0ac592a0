# round 4: the rhs in cell order (pencil + gather): parity files that read the
# rhs, the three-way assembly probe, the B^T tasks-per-wave variants, SQ
# counters of the assembly kernels
set -o pipefail
OUT=gpurun_out/r04l
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python3 -u tools/bt_rows_probe.py > $OUT/probe.json 2> $OUT/probe.err || { echo "probe failed"; tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.json
timeout -k 10 900 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_parity_gpu.py tests/test_cube.py tests/test_distributed_upload.py tests/test_refine6.py \
  tests/test_golden.py "tests/test_multi_rank.py::test_group_time_step_matches_single_gpu" \
  tests/test_multi_rank.py::test_group_bench_sequence_8_ranks tests/test_multi_rank.py::test_group_rank_without_pressure_rows \
  > $OUT/tests.log 2>&1 || { echo "tests failed"; grep -E "PASSED|FAILED|Error" $OUT/tests.log | head -80; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python3 -u tools/variant_probe.py > $OUT/variants.json 2> $OUT/variants.err || { echo "variants failed"; tail -5 $OUT/variants.err; exit 1; }
cat $OUT/variants.json
echo ALLOK
