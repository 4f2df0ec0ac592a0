# round 4: the new GPU tests first (repeated operator-form assembly, hand-off
# timeout rerun, zero-pressure-row rank, RCCL self-peer halo, 8 ranks at r=4,
# refine 6), then the whole GPU suite
set -o pipefail
OUT=gpurun_out/r04a
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_multi_rank.py::test_halo_exchange_round_trip_self_peer \
  "tests/test_parity_gpu.py::test_repeated_operator_form_assembly_matches_oracle" \
  "tests/test_parity_gpu.py::test_handoff_timeout_reruns_on_multi_launch_kernels" \
  tests/test_cube.py::test_cube_repeated_operator_form_assembly \
  tests/test_multi_rank.py::test_group_rank_without_pressure_rows \
  tests/test_multi_rank.py::test_group_8_ranks_refine4_fixed_inner \
  tests/test_refine6.py > $OUT/new_tests.log 2>&1 || { echo "new tests failed"; tail -60 $OUT/new_tests.log; exit 1; }
grep -E "PASSED|FAILED|scatter info|device memory|residual reduction" $OUT/new_tests.log | tail -40
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
echo ALLOK
