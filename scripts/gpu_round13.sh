set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu13.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_mine13.json 2> gpurun_out/bench_mine13.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/bench_verify13.json 2> gpurun_out/bench_verify13.err || exit $?
timeout -k 10 300 python scripts/node_soak.py --seconds 90 --out gpurun_out/soak13.json > gpurun_out/soak13.log 2>&1; echo "soak rc=$?"
