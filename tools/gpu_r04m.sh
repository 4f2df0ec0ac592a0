# round 4: B^T task kernel v2 (constraint loads in phase 1, packed destination
# scan) against the previous kernel (bitwise, assembly time), its SQ counters,
# then the bench with the rhs in cell order
set -o pipefail
OUT=gpurun_out/r04m
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/variant_probe.py > $OUT/variants.json 2> $OUT/variants.err || { echo "variants failed"; tail -5 $OUT/variants.err; exit 1; }
cat $OUT/variants.json
rm -rf /tmp/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --kernel-include-regex "k_bt_tasks" --output-format csv -d /tmp/pmc -o pmc -- python3 $GRAFT_REPO_ROOT/tools/bt_rows_probe.py > $OUT/sq.log 2>&1 || { echo "sq failed"; tail -5 $OUT/sq.log; exit 1; }
find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/sq.csv \;
python3 - <<'PY'
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open("gpurun_out/r04m/sq.csv")):
    acc[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['gmres_inner_iter_per_s'], d['phase_ms'], d['roofline']['frac'], d['roofline_matrix_free']['frac'])"
echo ALLOK
