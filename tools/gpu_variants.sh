set -o pipefail
mkdir -p gpurun_out/r04t
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REPS=${REPS:-6} timeout -k 10 300 python3 -u tools/variant_probe.py > gpurun_out/r04t/store_variants.json 2> gpurun_out/r04t/store_variants.err || { tail -5 gpurun_out/r04t/store_variants.err; exit 1; }
cat gpurun_out/r04t/store_variants.json
timeout -k 10 200 python3 -u tools/env_probe.py DCP_ASM_OVERLAP 0 1 2 0 > gpurun_out/r04t/overlap.json 2> gpurun_out/r04t/overlap.err || { tail -5 gpurun_out/r04t/overlap.err; exit 1; }
cat gpurun_out/r04t/overlap.json
DCP_ASM_OVERLAP=1 REPS=${REPS:-6} timeout -k 10 300 python3 -u tools/variant_probe.py > gpurun_out/r04t/store_variants_ov1.json 2> gpurun_out/r04t/store_variants_ov1.err || { tail -5 gpurun_out/r04t/store_variants_ov1.err; exit 1; }
cat gpurun_out/r04t/store_variants_ov1.json
