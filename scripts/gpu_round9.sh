set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu9.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/bench_verify9.json 2> gpurun_out/bench_verify9.err; echo "verify rc=$?"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof9 -o verify --output-format csv -- python3 bench.py --mode verify --steps 2 --warmup 1 > gpurun_out/prof9.log 2>&1; echo "prof rc=$?"
