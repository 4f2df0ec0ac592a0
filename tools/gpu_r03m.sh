set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_multi_rank.py tests/test_renumber.py -k "sstep or dealii or dealii_93" > gpurun_out/r03m_sstep_tests.log 2>&1 || { echo "sstep tests failed"; tail -40 gpurun_out/r03m_sstep_tests.log; exit 1; }
tail -3 gpurun_out/r03m_sstep_tests.log
for gs in classical2 sstep; do
  VAR=none GS=$gs REPS=4 timeout -k 10 200 python3 -u tools/inner_probe.py > gpurun_out/r03m_inner_$gs.json 2>&1 || { echo "probe $gs failed"; tail -5 gpurun_out/r03m_inner_$gs.json; exit 1; }
  cat gpurun_out/r03m_inner_$gs.json
done

GS=sstep VAR=none REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03m_prof -o sstep -- python3 -u tools/inner_probe.py > gpurun_out/r03m_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/r03m_prof.log; exit 1; }
echo ALLOK
