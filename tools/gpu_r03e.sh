set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/dcgs_timing.py > gpurun_out/r03e_dcgs_timing.json 2>&1 || { echo "timing failed"; tail -5 gpurun_out/r03e_dcgs_timing.json; exit 1; }
cat gpurun_out/r03e_dcgs_timing.json | cut -c1-600
R=6 timeout -k 10 600 python3 -u tools/r6_probe.py > gpurun_out/r03e_r6_probe.log 2>&1 || { echo "r6 probe failed"; tail -3 gpurun_out/r03e_r6_probe.log; exit 1; }
tail -1 gpurun_out/r03e_r6_probe.log | cut -c1-300
timeout -k 10 900 python3 -u bench.py --refine 6 --steps 1 --warmup 1 --no-cpu-baseline --no-converging-leg --gram-schmidt dcgs2 > gpurun_out/r03e_bench_r6.json 2> gpurun_out/r03e_bench_r6.err || { echo "bench r6 failed"; tail -5 gpurun_out/r03e_bench_r6.err; exit 1; }
echo ALLOK
