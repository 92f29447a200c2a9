set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu33.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke33.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_mine33.json 2> gpurun_out/bench_mine33.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 > gpurun_out/bench_verify33.json 2> gpurun_out/bench_verify33.err || exit $?
timeout -k 10 500 python bench.py --mode sync --steps 5 --warmup 1 > gpurun_out/bench_sync33.json 2> gpurun_out/bench_sync33.err || exit $?
