# round 4: S formation rewrite (old vs new, bitwise, time), then the whole GPU
# suite, smoke and the r=5 bench
set -o pipefail
OUT=gpurun_out/r04n
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u tools/schur_form_probe.py > $OUT/schur_form.json 2> $OUT/schur_form.err || { echo "schur probe failed"; tail -5 $OUT/schur_form.err; exit 1; }
cat $OUT/schur_form.json
timeout -k 10 800 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['gmres_inner_iter_per_s'], d['phase_ms'], d['roofline']['frac'], d['roofline_matrix_free']['frac'])"
echo ALLOK
