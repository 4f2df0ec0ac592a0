set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "matrix_free or operator or cube or multi_rank or full_solve" > gpurun_out/r03q_mf_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03q_mf_tests.log; exit 1; }
tail -2 gpurun_out/r03q_mf_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03q_mfprobe -o run -- python3 tools/mf_probe.py > gpurun_out/r03q_mf_probe.log 2>&1 || { echo "mf probe failed"; tail -5 gpurun_out/r03q_mf_probe.log; exit 1; }
cat gpurun_out/r03q_mf_probe.log | tail -2
grep -E "k_mf_pencil|k_mf_gather" gpurun_out/r03q_mfprobe/run_kernel_stats.csv | cut -c1-60,150-260
timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-converging-leg > gpurun_out/r03q_bench.json 2> gpurun_out/r03q_bench.err || { echo "bench failed"; tail -5 gpurun_out/r03q_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03q_bench.json')); print(d['ms_per_step'], d['roofline_matrix_free']['avg_apply_ms'], d['roofline_matrix_free']['frac'], d['roofline_matrix_free']['velocity_block']['avg_apply_ms'])"

timeout -k 10 600 python3 -u bench.py --refine 6 --steps 1 --warmup 1 --no-cpu-baseline --no-converging-leg > gpurun_out/r03q_bench_r6.json 2> gpurun_out/r03q_bench_r6.err || { echo "bench r6 failed"; tail -8 gpurun_out/r03q_bench_r6.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03q_bench_r6.json')); print(d['value'], d['ms_per_step'], d['gmres_inner_iter_per_s'], d['roofline']['frac'], d['device_mem_gb'], d['setup_s']); print([(o['gram_schmidt'], o['solve_nse_ms']) for o in d['other_gram_schmidt']])"
echo ALLOK
