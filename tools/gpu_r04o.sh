# round 4: matrix-free pencil, per-wave (ungrouped) vs per-workgroup group
# indexing at one wave (kernel times under rocprofv3, two runs each)
set -o pipefail
OUT=gpurun_out/r04o
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for run in 1 2; do
  for V in a_ungrouped b_grouped; do
    rm -rf /tmp/prof
    VAR=$V R=5 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o mf -- python3 -u tools/mf_probe.py > $OUT/mf_${V}_$run.json 2> $OUT/mf_${V}_$run.err || { echo "mf probe $V failed"; tail -5 $OUT/mf_${V}_$run.err; exit 1; }
    f=$(find /tmp/prof -name "*kernel_stats.csv" | head -1)
    cp "$f" $OUT/mf_${V}_${run}_kernel_stats.csv
    echo "$V run $run: $(cut -c1-200 $OUT/mf_${V}_$run.json)"
    grep -E "k_mf_pencil<true, true|k_mf_gather<true" $OUT/mf_${V}_${run}_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
  done
done
echo ALLOK
