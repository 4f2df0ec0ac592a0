set -o pipefail
mkdir -p gpurun_out/r03ag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03ag
GS=sstep timeout -k 10 400 python3 -u tools/inner_probe.py > $OUT/inner.log 2>&1 || { echo "inner probe failed"; tail -5 $OUT/inner.log; exit 1; }
cut -c1-300 $OUT/inner.log
for V in base nt2; do
  VAR=$V GS=sstep REPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$V -o inner -- python3 -u tools/inner_probe.py > $OUT/prof_$V.log 2>&1 || { echo "prof $V failed"; tail -5 $OUT/prof_$V.log; exit 1; }
  grep -E "k_sell_spmv|k_sstep_block<28>|k_sstep_block<4>" $OUT/prof_$V/inner_kernel_stats.csv | cut -d, -f1-4 | cut -c1-40,150-260
done
echo ALLOK
