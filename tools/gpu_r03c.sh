set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_multi_rank.py -m gpu -v --timeout 300 --timeout-method thread -k "DCGS2 or dcgs2 or cgs2 or forced" > gpurun_out/r03c_gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r03c_gputest.log; exit 1; }
tail -3 gpurun_out/r03c_gputest.log
for gs in dcgs2 classical2; do
  R=5 REPS=3 GS=$gs timeout -k 10 300 python3 tools/inner_probe.py > gpurun_out/r03c_inner_$gs.json 2>&1 || { echo "probe $gs failed"; tail -5 gpurun_out/r03c_inner_$gs.json; exit 1; }
  cat gpurun_out/r03c_inner_$gs.json
done
R=5 REPS=2 GS=dcgs2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03c_prof -o run -- python3 tools/inner_probe.py > gpurun_out/r03c_prof.log 2>&1 || { echo "prof failed"; exit 1; }
echo ALLOK
