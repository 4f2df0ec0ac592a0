set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_multi_rank.py -k "sstep" > gpurun_out/r03t_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03t_tests.log; exit 1; }
tail -1 gpurun_out/r03t_tests.log
for R in 4 5 6; do
  R=$R timeout -k 10 120 python3 -u tools/sstep_multi_probe.py >> gpurun_out/r03t_multi.log 2>&1 || { echo "R=$R failed or timed out"; tail -5 gpurun_out/r03t_multi.log; exit 1; }
  tail -1 gpurun_out/r03t_multi.log
done
echo ALLOK
