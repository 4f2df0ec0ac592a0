set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_schur_solver.py -m gpu > gpurun_out/r03i_gpu.log 2>&1; tail -2 gpurun_out/r03i_gpu.log
timeout -k 10 300 python3 -u tools/dcgs_timing.py > gpurun_out/r03i_dcgs_timing.json 2>&1 || { echo "timing failed"; tail -5 gpurun_out/r03i_dcgs_timing.json; exit 1; }
cut -c1-800 gpurun_out/r03i_dcgs_timing.json
R=6 timeout -k 10 500 python3 -u tools/r6_probe.py > gpurun_out/r03i_r6_probe.log 2>&1 || { echo "r6 probe failed"; tail -3 gpurun_out/r03i_r6_probe.log; exit 1; }
tail -2 gpurun_out/r03i_r6_probe.log | cut -c1-400
echo ALLOK
