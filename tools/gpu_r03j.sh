set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest -v --timeout 150 --timeout-method thread tests/test_parity_gpu.py -m gpu -k "sstep or cgs2_cycle" > gpurun_out/r03j_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r03j_gpu.log
[ $rc -le 1 ] || { echo "pytest aborted rc=$rc"; exit 1; }
for gs in classical2 sstep; do
  GS=$gs REPS=4 timeout -k 10 200 python3 -u tools/inner_probe.py > gpurun_out/r03j_inner_$gs.json 2>&1 || { echo "probe $gs failed"; tail -5 gpurun_out/r03j_inner_$gs.json; exit 1; }
  cat gpurun_out/r03j_inner_$gs.json
done
echo ALLOK
