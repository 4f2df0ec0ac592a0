set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 ./tools/vecread_probe > gpurun_out/r03d_vecread.txt 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --durations=10 > gpurun_out/r03d_gputest.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/r03d_gputest.log | head -20; tail -5 gpurun_out/r03d_gputest.log; exit 1; }
tail -2 gpurun_out/r03d_gputest.log
R=6 timeout -k 10 600 python3 -u tools/r6_probe.py > gpurun_out/r03d_r6_probe.log 2>&1 || { echo "r6 probe failed"; tail -5 gpurun_out/r03d_r6_probe.log; exit 1; }
tail -1 gpurun_out/r03d_r6_probe.log
timeout -k 10 900 python3 -u bench.py --refine 6 --steps 1 --warmup 1 --no-cpu-baseline --no-converging-leg --gram-schmidt dcgs2 > gpurun_out/r03d_bench_r6.json 2> gpurun_out/r03d_bench_r6.err || { echo "bench r6 failed"; tail -5 gpurun_out/r03d_bench_r6.err; exit 1; }
echo ALLOK
