# round 4: kernel split of the B^T-by-rows assembly (rocprof of the probe)
set -o pipefail
OUT=gpurun_out/r04d
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o probe -- python3 -u tools/bt_rows_probe.py > $OUT/probe_prof.json 2> $OUT/probe_prof.err || { echo "prof failed"; tail -5 $OUT/probe_prof.err; exit 1; }
cat $OUT/probe_prof.json
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/probe_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04d/probe_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["TotalDurationNs"]) / 1e6, 2), "ms")
PY
echo ALLOK
