set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 --from-mempool > gpurun_out/bench_verify26_mp.json 2> gpurun_out/bench_verify26_mp.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 > gpurun_out/bench_verify26.json 2> gpurun_out/bench_verify26.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 --from-mempool --ledger /tmp/upow_bench_ledger > gpurun_out/bench_verify26_mp_file.json 2> gpurun_out/bench_verify26_mp_file.err || exit $?
rm -rf /tmp/upow_bench_ledger
