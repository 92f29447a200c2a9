set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for k in 1 2; do
timeout -k 10 400 python bench.py --mode verify --steps 6 --warmup 2 --ledger /tmp/upow_bench_ledger > gpurun_out/bench_verify23_bg$k.json 2> gpurun_out/bench_verify23_bg$k.err || exit $?
rm -rf /tmp/upow_bench_ledger
UPOW_WAL_CHECKPOINT_THREAD=0 timeout -k 10 400 python bench.py --mode verify --steps 6 --warmup 2 --ledger /tmp/upow_bench_ledger > gpurun_out/bench_verify23_fg$k.json 2> gpurun_out/bench_verify23_fg$k.err || exit $?
rm -rf /tmp/upow_bench_ledger
done
