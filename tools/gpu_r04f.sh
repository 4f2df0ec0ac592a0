# round 4: new assembly probe (B^T row tasks + two-cells-per-wave rhs), the
# new GPU tests, the whole GPU suite, smoke, bench r=5 and its kernel statistics
set -o pipefail
OUT=gpurun_out/r04f
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 240 python3 -u tools/bt_rows_probe.py > $OUT/probe.json 2> $OUT/probe.err || { echo "probe failed"; tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.json
timeout -k 10 900 python3 -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_multi_rank.py::test_halo_exchange_round_trip_self_peer \
  "tests/test_parity_gpu.py::test_repeated_operator_form_assembly_matches_oracle" \
  "tests/test_parity_gpu.py::test_handoff_timeout_reruns_on_multi_launch_kernels" \
  tests/test_cube.py::test_cube_repeated_operator_form_assembly \
  tests/test_multi_rank.py::test_group_rank_without_pressure_rows \
  tests/test_multi_rank.py::test_group_8_ranks_refine4_fixed_inner \
  tests/test_multi_rank.py::test_group_matrix_powers_bitwise \
  tests/test_driver.py tests/test_refine6.py > $OUT/new_tests.log 2>&1 || { echo "new tests failed"; tail -60 $OUT/new_tests.log; exit 1; }
grep -E "PASSED|FAILED|scatter info|device memory|residual reduction" $OUT/new_tests.log | tail -40
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['gmres_inner_iter_per_s'], d['phase_ms'], d['roofline']['frac'], d['roofline_matrix_free']['frac'])"
echo ALLOK
