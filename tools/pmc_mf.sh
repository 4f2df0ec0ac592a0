# PMC passes over the matrix-free probe (tools/mf_probe.py): one rocprofv3 run
# per counter group, kernel-trace only, results summarised on the box.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcmf
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KRE=${KRE:-"k_mf_pencil|k_mf_gather"}
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  rm -rf /tmp/pmc
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex "$KRE" --output-format csv -d /tmp/pmc -o pmc -- python3 $GRAFT_REPO_ROOT/tools/mf_probe.py > $OUT/probe_$i.log 2>&1 || exit $?
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/g$i.csv \;
done
python3 - <<'PY'
import csv, glob, json, os, collections
out = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/pmcmf"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(out + "/g*.csv")):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
res = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}
json.dump(res, open(out + "/summary.json", "w"), indent=1)
PY
rm -f $OUT/g*.csv
