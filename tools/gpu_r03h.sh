set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_parity_gpu_2d.py tests/test_temperature_q2.py tests/test_distributed_upload.py tests/test_schur_solver.py -m gpu > gpurun_out/r03h_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03h_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest aborted rc=$rc"; exit 1; }
timeout -k 10 300 python3 -u tools/dcgs_timing.py > gpurun_out/r03h_dcgs_timing.json 2>&1 || { echo "timing failed"; tail -5 gpurun_out/r03h_dcgs_timing.json; exit 1; }
cut -c1-600 gpurun_out/r03h_dcgs_timing.json
R=6 timeout -k 10 450 python3 -u tools/r6_probe.py > gpurun_out/r03h_r6_probe.log 2>&1 || { echo "r6 probe failed"; tail -3 gpurun_out/r03h_r6_probe.log; exit 1; }
tail -1 gpurun_out/r03h_r6_probe.log | cut -c1-300
echo ALLOK
