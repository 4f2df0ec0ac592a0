set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r03n_gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/r03n_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r03n_gpu_tests.log
for gs in classical2 sstep; do
  VAR=none GS=$gs REPS=4 timeout -k 10 200 python3 -u tools/inner_probe.py > gpurun_out/r03n_inner_$gs.json 2>&1 || { echo "probe $gs failed"; tail -5 gpurun_out/r03n_inner_$gs.json; exit 1; }
  cat gpurun_out/r03n_inner_$gs.json
done
echo ALLOK
