set -u
OUT=gpurun_out/pmc_asm; mkdir -p $OUT
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d /tmp/pmc -o pmc -- python3 tools/asm_probe.py > $OUT/$ctr.log 2>&1 || exit 1
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/${ctr}.csv \;
done
rm -rf /tmp/kt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/kt -o kt -- python3 tools/asm_probe.py > $OUT/kt.log 2>&1 || exit 1
find /tmp/kt -name "*kernel_trace*.csv" -exec cp {} $OUT/kernel_trace.csv \;
