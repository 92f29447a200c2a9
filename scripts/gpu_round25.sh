set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu25.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke25.log 2>&1 || exit $?
UPOW_TXCODEC_PROFILE=1 timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 > gpurun_out/bench_verify25.json 2> gpurun_out/bench_verify25.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 > gpurun_out/bench_verify25b.json 2> gpurun_out/bench_verify25b.err || exit $?
timeout -k 10 500 python bench.py --mode sync --steps 5 --warmup 1 > gpurun_out/bench_sync25.json 2> gpurun_out/bench_sync25.err || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_mine25.json 2> gpurun_out/bench_mine25.err || exit $?
