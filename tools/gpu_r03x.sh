set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_golden.py tests/test_temperature_q2.py tests/test_multi_rank.py tests/test_driver.py tests/test_distributed_upload.py > gpurun_out/r03x_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03x_tests.log; exit 1; }
tail -2 gpurun_out/r03x_tests.log
for v in 0 1; do
  DCP_ASM_CELL_BLOCK=$v timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-converging-leg > gpurun_out/r03x_bench_$v.json 2> gpurun_out/r03x_bench_$v.err || { echo "bench $v failed"; tail -5 gpurun_out/r03x_bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03x_bench_$v.json')); print('cell_block=$v', d['value'], d['phase_ms']['assemble_nse_ms'], d['ms_per_step'])"
done
echo ALLOK
