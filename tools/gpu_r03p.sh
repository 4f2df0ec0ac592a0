set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u bench.py --refine 6 --steps 1 --warmup 1 --no-cpu-baseline --no-converging-leg > gpurun_out/r03p_bench_r6.json 2> gpurun_out/r03p_bench_r6.err || { echo "bench r6 failed"; tail -5 gpurun_out/r03p_bench_r6.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03p_bench_r6.json')); print(d['value'], d['ms_per_step'], d['gmres_inner_iter_per_s'], d['roofline']['frac'], d['device_mem_gb'], d['setup_s']); print([(o['gram_schmidt'], o['solve_nse_ms']) for o in d['other_gram_schmidt']])"
timeout -k 10 300 python3 -u -m pytest -x -v -s --timeout 250 --timeout-method thread -m gpu tests/test_golden.py -k "r3_matches" > gpurun_out/r03p_r3.log 2>&1 || { echo "r3 tests failed"; tail -30 gpurun_out/r03p_r3.log; exit 1; }
grep "r3 step" gpurun_out/r03p_r3.log
echo ALLOK
