set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu4.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/bench_verify4.log 2>&1; echo "verify rc=$?"
timeout -k 10 200 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_mine4.log 2>&1; echo "mine rc=$?"
