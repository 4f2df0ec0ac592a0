set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_golden.py tests/test_temperature_q2.py tests/test_driver.py tests/test_renumber.py > gpurun_out/r03aa_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r03aa_tests.log; exit 1; }
tail -2 gpurun_out/r03aa_tests.log
for v in 0 1; do
  DCP_ASM_PER_CELL=$v timeout -k 10 200 python3 -u tools/variant_probe.py > gpurun_out/r03aa_asm_$v.log 2>&1 || { echo "probe $v failed"; tail -5 gpurun_out/r03aa_asm_$v.log; exit 1; }
  echo "per_cell=$v"; cut -c1-110 gpurun_out/r03aa_asm_$v.log
done
echo ALLOK
