set -o pipefail
mkdir -p gpurun_out/r03ai
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03ai
for V in base gv2; do
  VAR=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$V -o mf -- python3 -u tools/mf_probe.py > $OUT/mf_$V.log 2>&1 || { echo "mf $V failed"; tail -5 $OUT/mf_$V.log; exit 1; }
  grep variant $OUT/mf_$V.log | cut -c1-400
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/prof_$V/mf_kernel_stats.csv')):
    if 'k_mf_pencil<true' in r['Name'] or 'k_mf_gather<true>' in r['Name']: print('$V', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 2))"
done
echo ALLOK
