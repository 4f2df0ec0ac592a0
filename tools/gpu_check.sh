#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 stats + PMC traffic probe.
# Every GPU step has its own time limit; a fault/abort/timeout stops the script.
set -u
OUT=gpurun_out
mkdir -p $OUT
ok() {  # continue only on success or an ordinary test failure (rc 1)
  local rc=$1; shift
  echo "$* rc=$rc" >> $OUT/steps.log
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after rc=$rc ($*)" >> $OUT/steps.log; exit $rc; fi
}
STEPS=${STEPS:-"pytest bench profile pmc"}
R=${R:-5}
for s in $STEPS; do
  case $s in
    pytest)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; ok $? pytest ;;
    bench)
      timeout -k 10 600 python bench.py --refine $R --steps ${K:-2} --warmup ${W:-1} > $OUT/bench.json 2> $OUT/bench.err; ok $? bench ;;
    profile)
      rm -rf /tmp/prof && mkdir -p $OUT/prof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o run \
        -- python3 bench.py --refine $R --steps 1 --warmup 0 --no-cpu-baseline > $OUT/prof/bench_profiled.json 2> $OUT/prof/rocprof.err
      rc=$?; find /tmp/prof -name "*stats*.csv" -exec cp {} $OUT/prof/ \; ; ok $rc profile ;;
    pmc)
      mkdir -p $OUT/pmc
      for ctr in FETCH_SIZE WRITE_SIZE; do
        rm -rf /tmp/pmc
        timeout -k 10 600 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "${PMC_KERNELS:-k_sell_spmv|k_nse_system|k_chain}" \
          --output-format csv -d /tmp/pmc -o pmc \
          -- python3 bench.py --refine $R --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc/probe_$ctr.json 2> $OUT/pmc/probe_$ctr.err
        rc=$?; find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/pmc/${ctr}.csv \; ; ok $rc pmc_$ctr
      done
      # summarise on the box: the per-dispatch CSVs exceed gpurun's copy-back cap
      python3 tools/pmc_summary.py $OUT/pmc "rocprofv3 --pmc <CTR> --kernel-trace --kernel-include-regex '${PMC_KERNELS:-k_sell_spmv|k_nse_system|k_chain}' -- python3 bench.py --refine $R --steps 1 --warmup 0 --no-cpu-baseline" $OUT/pmc/summary.json
      ok $? pmc_summary
      rm -f $OUT/pmc/*.csv ;;
  esac
done
echo done >> $OUT/steps.log
