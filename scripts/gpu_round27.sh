set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu27.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 > gpurun_out/bench_verify27.json 2> gpurun_out/bench_verify27.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 --from-mempool > gpurun_out/bench_verify27_mp.json 2> gpurun_out/bench_verify27_mp.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 --from-mempool --ledger /tmp/upow_bench_ledger > gpurun_out/bench_verify27_mp_file.json 2> gpurun_out/bench_verify27_mp_file.err || exit $?
rm -rf /tmp/upow_bench_ledger
