# round 4 final: the whole GPU suite, smoke, the default bench, its kernel
# statistics, PMC traffic of the assembly kernels the line cites
set -o pipefail
OUT=gpurun_out/${TAGR:-r04r}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['gmres_inner_iter_per_s'], d['phase_ms'], d['roofline']['frac'], d['roofline_matrix_free']['frac'])"
rm -rf /tmp/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o bench -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-converging-leg > $OUT/bench_prof.json 2> $OUT/bench_prof.err || { echo "bench prof failed"; tail -5 $OUT/bench_prof.err; exit 1; }
f=$(find /tmp/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $OUT/bench_kernel_stats.csv
TAG=${TAGR:-r04r}_pmc_asm REGEX="k_bt_tasks|k_bt_coltab|k_mf_pencil|k_mf_gather|k_nse_rhs_halfwave|k_con_gather" bash tools/pmc_pass.sh tools/asm_probe.py || { echo "pmc asm failed"; exit 1; }

timeout -k 10 200 python3 -u tools/bt_slots_probe.py > $OUT/bt_slots.json 2> $OUT/bt_slots.err || { echo "bt slots probe failed"; tail -5 $OUT/bt_slots.err; exit 1; }
cat $OUT/bt_slots.json
echo ALLOK
