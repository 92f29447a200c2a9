set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu20.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 > gpurun_out/bench_verify20.json 2> gpurun_out/bench_verify20.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 > gpurun_out/bench_verify20b.json 2> gpurun_out/bench_verify20b.err || exit $?
timeout -k 10 300 python scripts/p256_throughput.py > gpurun_out/p256_20.txt 2>&1 || exit $?
