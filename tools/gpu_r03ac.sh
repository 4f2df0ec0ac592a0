set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03ac_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03ac_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03ac_gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03ac_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/r03ac_smoke.log; exit 1; }
tail -1 gpurun_out/r03ac_smoke.log
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03ac_bench.json 2> gpurun_out/r03ac_bench.err || { echo "bench failed"; tail -5 gpurun_out/r03ac_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03ac_bench.json')); print(d['value'], d['ms_per_step'], d['gmres_inner_iter_per_s'], d['roofline']['frac'], d['roofline_matrix_free']['frac']); print(d['assembly_with_velocity_block']['roofline']); print(d['T_assembly'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03ac_prof -o bench -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-converging-leg > gpurun_out/r03ac_bench_prof.json 2> gpurun_out/r03ac_bench_prof.err || { echo "bench prof failed"; tail -5 gpurun_out/r03ac_bench_prof.err; exit 1; }
head -8 gpurun_out/r03ac_prof/bench_kernel_stats.csv | cut -c1-150
echo ALLOK
