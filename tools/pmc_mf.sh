set -u
mkdir -p gpurun_out/pmcmf
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-trace --kernel-include-regex "k_mf_stokes" --output-format csv -d /tmp/pmc -o pmc -- python3 tools/mf_probe.py > gpurun_out/pmcmf/probe_$ctr.log 2>&1 || exit $?
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} gpurun_out/pmcmf/${ctr}.csv \;
done
