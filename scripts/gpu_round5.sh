set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu5.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/bench_verify5.log 2>&1; echo "verify rc=$?"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o verify --output-format csv -- python3 bench.py --mode verify --steps 2 --warmup 1 > gpurun_out/prof5.log 2>&1; echo "prof rc=$?"
timeout -k 10 300 python scripts/p256_throughput.py > gpurun_out/p256_tp5.log 2>&1; echo "tp rc=$?"
