# round 4: assembly variants (bitwise / time), kernel split, parity files;
# (earlier: B^T task kernel, per-slot vertex table (no scan over all (slot,
# vertex) pairs) against the scan (bitwise, assembly time); kernel split;
# parity files
set -o pipefail
OUT=gpurun_out/r04q
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/variant_probe.py > $OUT/variants.json 2> $OUT/variants.err || { echo "variants failed"; tail -5 $OUT/variants.err; exit 1; }
cat $OUT/variants.json
rm -rf /tmp/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o probe -- python3 -u tools/bt_rows_probe.py > $OUT/probe.json 2> $OUT/probe.err || { echo "probe failed"; tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.json
f=$(find /tmp/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/probe_kernel_stats.csv
grep -E "k_bt_tasks|k_mf_pencil<false|k_mf_gather<false|k_nse_rhs_halfwave|k_bt_coltab" $OUT/probe_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_multi_rank.py::test_group_time_step_matches_single_gpu tests/test_cube.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
echo ALLOK
