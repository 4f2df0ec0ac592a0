# Round-6 measurement set (run on the GPU box from the repo root):
# 1. rocprofv3 --kernel-trace --stats of the default refine-5 step alone
#    (no converging refine-3 leg, no other Gram-Schmidt legs), the trace
#    summarised with tools/trace_summary.py (early-exit launches split off);
# 2. FETCH_SIZE / WRITE_SIZE passes over the matrix-free apply
#    (tools/mf_probe.py, r=5), summarised with tools/pmc_summary.py.
set -u
TAG=${TAG:-r06n}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-converging-leg --no-other-gs"
rm -rf /tmp/kt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kt -o run -- $CMD > $OUT/bench_traced.log 2>&1 || exit 1
cp /tmp/kt/run_kernel_stats.csv $OUT/kernel_stats.csv
python3 tools/trace_summary.py /tmp/kt/run_kernel_trace.csv $OUT/trace_r5.json "rocprofv3 --kernel-trace --stats -- $CMD" || exit 1
rm -rf /tmp/kt
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc
  R=5 VAR=none timeout -s KILL 180 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "k_mf_pencil|k_mf_gather" --output-format csv -d /tmp/pmc -o pmc -- python3 tools/mf_probe.py > $OUT/pmc_mf_$ctr.log 2>&1 || exit 1
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/$ctr.csv \;
done
python3 tools/pmc_summary.py $OUT "rocprofv3 --pmc <CTR> --kernel-trace --kernel-include-regex 'k_mf_pencil|k_mf_gather' -- python3 tools/mf_probe.py (R=5)" $OUT/pmc_mf_r5.json || exit 1
rm -f $OUT/FETCH_SIZE.csv $OUT/WRITE_SIZE.csv
echo done
