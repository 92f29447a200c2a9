set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu12.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/bench_verify12.json 2> gpurun_out/bench_verify12.err; echo "verify rc=$?"
timeout -k 10 300 python bench.py > gpurun_out/bench_mine12.json 2> gpurun_out/bench_mine12.err; echo "mine rc=$?"
