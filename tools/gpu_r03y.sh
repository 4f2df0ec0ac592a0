set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u tools/variant_probe.py > gpurun_out/r03y_variants.log 2>&1 || { echo "variants failed"; tail -5 gpurun_out/r03y_variants.log; exit 1; }
cat gpurun_out/r03y_variants.log | cut -c1-120
echo ALLOK
