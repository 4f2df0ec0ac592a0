set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03o_bench.json 2> gpurun_out/r03o_bench.err || { echo "bench failed"; tail -5 gpurun_out/r03o_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03o_bench.json')); print(d['value'], d['ms_per_step'], d['gmres_inner_iter_per_s'], d['roofline']['frac'], d['roofline']['traffic']); print(d.get('converging_step')); print([(o['gram_schmidt'], o['solve_nse_ms']) for o in d['other_gram_schmidt']])"
GS=sstep VAR=none REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03o_probe -o sstep -- python3 -u tools/inner_probe.py > gpurun_out/r03o_probe.log 2>&1 || { echo "probe prof failed"; tail -5 gpurun_out/r03o_probe.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03o_prof -o bench -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-converging-leg > gpurun_out/r03o_bench_prof.json 2> gpurun_out/r03o_bench_prof.err || { echo "bench prof failed"; tail -5 gpurun_out/r03o_bench_prof.err; exit 1; }
echo ALLOK
