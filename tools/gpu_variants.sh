set -o pipefail
mkdir -p gpurun_out/r04t
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/variant_probe.py > gpurun_out/r04t/store_variants.json 2> gpurun_out/r04t/store_variants.err || { tail -5 gpurun_out/r04t/store_variants.err; exit 1; }
cat gpurun_out/r04t/store_variants.json
