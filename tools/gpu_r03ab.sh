set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_multi_rank.py -k "one_rank_rccl" > gpurun_out/r03ab_rccl.log 2>&1 || { echo "rccl tests failed"; tail -30 gpurun_out/r03ab_rccl.log; exit 1; }
tail -2 gpurun_out/r03ab_rccl.log
OUT=gpurun_out/r03ab_pmc; mkdir -p $OUT
for ctr in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d /tmp/pmc -o pmc -- python3 tools/asm_probe.py > $OUT/$ctr.log 2>&1 || { echo "pmc $ctr failed"; tail -3 $OUT/$ctr.log; exit 1; }
  find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/${ctr}.csv \;
done
python3 tools/pmc_summary.py $OUT "rocprofv3 --pmc <CTR> --kernel-trace -- python3 tools/asm_probe.py (R=5)" gpurun_out/r03ab_pmc_asm_wave.json
python3 -c "
import json; d=json.load(open('gpurun_out/r03ab_pmc_asm_wave.json'))
for k,v in d['traffic_bytes'].items():
    if 'operator' in k or 'k_nse' in k: print(k[:70], round(v/1e6,1), 'MB/dispatch')"
echo ALLOK
