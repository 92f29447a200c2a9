set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu29.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --mode verify --steps 3 --warmup 1 --object-path > gpurun_out/bench_verify29_obj.json 2> gpurun_out/bench_verify29_obj.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 > gpurun_out/bench_verify29.json 2> gpurun_out/bench_verify29.err || exit $?
