set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_mine21.json 2> gpurun_out/bench_mine21.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 --ledger /tmp/upow_bench_ledger > gpurun_out/bench_verify21_file.json 2> gpurun_out/bench_verify21_file.err || exit $?
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 > gpurun_out/bench_verify21_mem.json 2> gpurun_out/bench_verify21_mem.err || exit $?
rm -rf /tmp/upow_bench_ledger
