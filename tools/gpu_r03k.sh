set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for gs in classical2 sstep; do
  VAR=none GS=$gs REPS=4 timeout -k 10 200 python3 -u tools/inner_probe.py > gpurun_out/r03k_inner_$gs.json 2>&1 || { echo "probe $gs failed"; tail -5 gpurun_out/r03k_inner_$gs.json; exit 1; }
  cat gpurun_out/r03k_inner_$gs.json
done
timeout -k 10 600 python3 -u bench.py --steps 3 --warmup 1 --gram-schmidt sstep --no-cpu-baseline > gpurun_out/r03k_bench_sstep.json 2> gpurun_out/r03k_bench_sstep.err || { echo "bench failed"; tail -5 gpurun_out/r03k_bench_sstep.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03k_bench_sstep.json')); print(d['ms_per_step'], d['gmres_inner_iter_per_s'], d['schur_gmres_inner_iterations'], d['fgmres_outer_iterations']); print(d.get('converging_step')); print([ (o['gram_schmidt'], o['solve_nse_ms'], o['gmres_inner_iter_per_s']) for o in d['other_gram_schmidt']])"
echo ALLOK
