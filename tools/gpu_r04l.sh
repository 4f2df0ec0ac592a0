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
timeout -k 10 300 python3 -u tools/mf_probe.py > $OUT/mf_variants.json 2> $OUT/mf_variants.err || { echo "mf probe failed"; tail -5 $OUT/mf_variants.err; exit 1; }
cat $OUT/mf_variants.json
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1)); rm -rf /tmp/pmc
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex "k_bt_tasks|k_mf_pencil|k_mf_gather|k_nse_rhs_halfwave" --output-format csv -d /tmp/pmc -o pmc -- python3 $GRAFT_REPO_ROOT/tools/bt_rows_probe.py > $OUT/sq_$i.log 2>&1 || { echo "sq pass $i failed"; tail -5 $OUT/sq_$i.log; exit 1; }
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/sq_g$i.csv \;
done
python3 - <<'PY'
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for g in (1, 2):
    for r in csv.DictReader(open(f"gpurun_out/r04l/sq_g{g}.csv")):
        acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
echo ALLOK
