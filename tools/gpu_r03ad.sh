set -o pipefail
mkdir -p gpurun_out/r03ad
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03ad
for T in 0 4096 100000; do
  DCP_ASM_SMALL_COLOUR=$T timeout -k 10 240 python3 -u tools/asm_probe.py > $OUT/asm_T$T.json 2>&1 || { echo "probe $T failed"; tail -5 $OUT/asm_T$T.json; exit 1; }
  echo "T=$T $(tail -1 $OUT/asm_T$T.json)"
done
for T in 0 4096; do
  DCP_ASM_SMALL_COLOUR=$T timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_T$T -o asm -- python3 -u tools/asm_probe.py > $OUT/trace_T$T.log 2>&1 || { echo "trace $T failed"; tail -5 $OUT/trace_T$T.log; exit 1; }
done
echo ALLOK
