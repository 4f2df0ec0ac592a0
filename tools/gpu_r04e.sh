# round 4: kernel split of the new assembly, then PMC traffic of the kernels
# the bench line cites (13-parameter k_sell_spmv, k_sstep_block, the assembly
# kernels, the matrix-free pencil / gather)
set -o pipefail
OUT=gpurun_out/r04e
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o probe -- python3 -u tools/bt_rows_probe.py > $OUT/probe_prof.json 2> $OUT/probe_prof.err || { echo "prof failed"; tail -5 $OUT/probe_prof.err; exit 1; }
cat $OUT/probe_prof.json
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/probe_kernel_stats.csv
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r04e/probe_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print(r["Name"][:80], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["TotalDurationNs"]) / 1e6, 2), "ms")
PY
TAG=r04e_pmc_asm REGEX="k_bt_tasks|k_bt_coltab|k_nse_operator_wave" bash tools/pmc_pass.sh tools/bt_rows_probe.py || { echo "pmc asm failed"; exit 1; }
R=5 REPS=2 GS=sstep TAG=r04e_pmc_inner REGEX="k_sell_spmv|k_sstep_block" bash tools/pmc_pass.sh tools/inner_probe.py || { echo "pmc inner failed"; exit 1; }
R=5 TAG=r04e_pmc_mf REGEX="k_mf_pencil|k_mf_gather" bash tools/pmc_pass.sh tools/mf_probe.py || { echo "pmc mf failed"; exit 1; }
for t in asm inner mf; do python3 -c "import json; d=json.load(open('gpurun_out/r04e_pmc_$t/summary.json')); print({k[:60]: round(v/1e6,1) for k, v in d['traffic_bytes'].items()})"; done
echo ALLOK
