# round 4: B^T tasks of 16 slots (two records per lane) against 8; assembly
# probe under rocprofv3 (kernel split) and the parity files that read B^T
set -o pipefail
OUT=gpurun_out/r04p
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf /tmp/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o probe -- python3 -u tools/bt_rows_probe.py > $OUT/probe.json 2> $OUT/probe.err || { echo "probe failed"; tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.json
f=$(find /tmp/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/probe_kernel_stats.csv
grep -E "k_bt_tasks|k_mf_pencil<false|k_mf_gather<false|k_nse_rhs_halfwave|k_bt_coltab" $OUT/probe_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
timeout -k 10 300 python3 -u tools/schur_form_probe.py > $OUT/schur_form.json 2> $OUT/schur_form.err || { echo "schur probe failed"; tail -5 $OUT/schur_form.err; exit 1; }
cat $OUT/schur_form.json
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_multi_rank.py::test_group_time_step_matches_single_gpu tests/test_refine6.py > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
echo ALLOK
