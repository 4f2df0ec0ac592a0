set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "assembled or operator_form or cube or golden or element" > gpurun_out/t_gputest.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/t_gputest.log; exit 1; }
timeout -k 10 300 python3 tools/variant_probe.py > gpurun_out/asm_var.txt 2>&1 || exit 1
echo ALLOK
