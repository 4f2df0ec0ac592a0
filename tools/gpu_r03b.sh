set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 ./tools/vecread_probe > gpurun_out/r03b_vecread.txt 2>&1 || { echo "probe failed"; exit 1; }
timeout -k 10 600 python3 bench.py --steps 2 --warmup 1 > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || { echo "bench failed"; tail -5 gpurun_out/r03b_bench.err; exit 1; }
echo ALLOK
