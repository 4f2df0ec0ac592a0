# round 4: kernel statistics of the r=5 bench and of the assembly probe, then
# PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the kernels the bench
# line cites: structured-column S SpMV + s-step block, the operator-form
# assembly (B^T row tasks, two-cells-per-wave rhs), the matrix-free apply
set -o pipefail
OUT=gpurun_out/r04j
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-converging-leg > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "bench prof failed"; tail -5 $OUT/bench_prof.err; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/bench_kernel_stats.csv
rm -rf $OUT/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/aprof -o probe -- python3 -u tools/bt_rows_probe.py > $OUT/probe_prof.json 2> $OUT/probe_prof.err || { echo "probe prof failed"; tail -5 $OUT/probe_prof.err; exit 1; }
f=$(find $OUT/aprof -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/probe_kernel_stats.csv
rm -rf $OUT/aprof
python3 - <<'PY'
import csv
for fn in ("bench", "probe"):
    rows = list(csv.DictReader(open(f"gpurun_out/r04j/{fn}_kernel_stats.csv")))
    print("==", fn)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
        print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us avg", round(float(r["TotalDurationNs"]) / 1e6, 2), "ms")
PY
R=5 REPS=2 GS=sstep VAR=none TAG=r04j_pmc_inner REGEX="k_sell_spmv|k_sstep_block" bash tools/pmc_pass.sh tools/inner_probe.py || { echo "pmc inner failed"; exit 1; }
TAG=r04j_pmc_asm REGEX="k_bt_tasks|k_bt_coltab|k_nse_rhs_halfwave|k_nse_operator_wave" bash tools/pmc_pass.sh tools/bt_rows_probe.py || { echo "pmc asm failed"; exit 1; }
R=5 VAR=none TAG=r04j_pmc_mf REGEX="k_mf_pencil|k_mf_gather" bash tools/pmc_pass.sh tools/mf_probe.py || { echo "pmc mf failed"; exit 1; }
for t in inner asm mf; do python3 -c "import json; d=json.load(open('gpurun_out/r04j_pmc_$t/summary.json')); print('$t', {k[:70]: round(v/1e6,2) for k, v in d['traffic_bytes'].items()})"; done
echo ALLOK
