# round 4: B^T task kernel tasks-per-wave variants (assembly time, bitwise),
# SQ counters of k_bt_tasks / k_nse_rhs_halfwave
set -o pipefail
OUT=gpurun_out/r04k
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/variant_probe.py > $OUT/variants.json 2> $OUT/variants.err || { echo "variants failed"; tail -5 $OUT/variants.err; exit 1; }
cat $OUT/variants.json
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"; do
  i=$((i+1)); rm -rf /tmp/pmc
  VAR=none timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex "k_bt_tasks|k_nse_rhs_halfwave" --output-format csv -d /tmp/pmc -o pmc -- python3 $GRAFT_REPO_ROOT/tools/bt_rows_probe.py > $OUT/sq_$i.log 2>&1 || { echo "sq pass $i failed"; tail -5 $OUT/sq_$i.log; exit 1; }
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/sq_g$i.csv \;
done
python3 - <<'PY'
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for g in (1, 2):
    for r in csv.DictReader(open(f"gpurun_out/r04k/sq_g{g}.csv")):
        acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
echo ALLOK
