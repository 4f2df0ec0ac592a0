set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for R in 5 6; do
  R=$R timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03u_prof$R -o p -- python3 -u tools/sstep_multi_probe.py > gpurun_out/r03u_multi$R.log 2>&1 || { echo "R=$R failed"; tail -5 gpurun_out/r03u_multi$R.log; exit 1; }
  grep "its" gpurun_out/r03u_multi$R.log
  head -14 gpurun_out/r03u_prof$R/p_kernel_stats.csv | cut -c1-160
done
echo ALLOK
