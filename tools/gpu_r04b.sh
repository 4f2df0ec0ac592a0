# round 4: B^T by rows -- probe (time + difference vs the cell scatter), the
# affected GPU tests, then kernel statistics of the probe
set -o pipefail
OUT=gpurun_out/r04b
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/bt_rows_probe.py > $OUT/probe.json 2> $OUT/probe.err || { echo "probe failed"; tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o probe -- python3 -u tools/bt_rows_probe.py > $OUT/probe_prof.json 2> $OUT/probe_prof.err || { echo "prof failed"; tail -5 $OUT/probe_prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/probe_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04b/probe_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg")
PY
echo ALLOK
