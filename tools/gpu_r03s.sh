set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GS=classical2 timeout -k 10 200 python3 -u tools/r6_probe.py > gpurun_out/r03s_r6_cgs2.log 2>&1 || { echo "cgs2 r6 probe failed"; tail -5 gpurun_out/r03s_r6_cgs2.log; }
tail -3 gpurun_out/r03s_r6_cgs2.log | cut -c1-400
GS=sstep timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03s_prof -o r6 -- python3 -u tools/r6_probe.py > gpurun_out/r03s_r6_sstep.log 2>&1 || { echo "sstep r6 probe failed"; tail -5 gpurun_out/r03s_r6_sstep.log; exit 1; }
tail -3 gpurun_out/r03s_r6_sstep.log | cut -c1-400
head -12 gpurun_out/r03s_prof/r6_kernel_stats.csv | cut -c1-200
echo ALLOK
