set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_multi_rank.py -k "one_rank_rccl" > gpurun_out/r03v_rccl.log 2>&1 || { echo "rccl test failed"; tail -30 gpurun_out/r03v_rccl.log; }
tail -4 gpurun_out/r03v_rccl.log
timeout -k 10 1000 python3 -u bench.py --refine 6 --steps 1 --warmup 0 --no-cpu-baseline --no-converging-leg > gpurun_out/r03v_bench_r6.json 2> gpurun_out/r03v_bench_r6.err || { echo "bench r6 failed"; tail -8 gpurun_out/r03v_bench_r6.err; exit 1; }
grep -v running gpurun_out/r03v_bench_r6.err
python3 -c "import json; d=json.load(open('gpurun_out/r03v_bench_r6.json')); print(d['value'], d['ms_per_step'], d['gmres_inner_iter_per_s'], d['roofline']['frac'], d['device_mem_gb'], d['setup_s']); print([(o['gram_schmidt'], o['solve_nse_ms']) for o in d['other_gram_schmidt']])"
echo ALLOK
