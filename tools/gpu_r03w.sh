set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 280 --timeout-method thread -m gpu tests/test_golden.py -k "r3_matches" > gpurun_out/r03w_r3.log 2>&1 || { echo "r3 tests failed"; tail -30 gpurun_out/r03w_r3.log; exit 1; }
grep -E "r3 step|passed|failed" gpurun_out/r03w_r3.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03w_bench.json 2> gpurun_out/r03w_bench.err || { echo "bench failed"; tail -5 gpurun_out/r03w_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03w_bench.json')); print(d['value'], d['ms_per_step'], d['gmres_inner_iter_per_s'], d['roofline']['frac'], d['roofline']['avg_apply_ms'], d['roofline_matrix_free']['frac']); print(d.get('converging_step')); print([(o['gram_schmidt'], o['solve_nse_ms']) for o in d['other_gram_schmidt']])"
echo ALLOK
