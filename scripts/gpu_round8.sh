set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu8.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/bench_verify8_native.json 2> gpurun_out/bench_verify8_native.err; echo "verify native rc=$?"
timeout -k 10 400 python bench.py --mode verify --steps 3 --warmup 1 --object-path > gpurun_out/bench_verify8_object.json 2> gpurun_out/bench_verify8_object.err; echo "verify object rc=$?"
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_mine8.json 2> gpurun_out/bench_mine8.err; echo "mine rc=$?"
