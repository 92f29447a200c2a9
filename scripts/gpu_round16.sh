set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu16.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 1 > gpurun_out/bench_verify16.json 2> gpurun_out/bench_verify16.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof16 -o verify --output-format csv -- python3 bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/prof16.log 2>&1; echo "prof rc=$?"
