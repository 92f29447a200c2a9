set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for k in 1 2; do
timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 --ledger /tmp/upow_bench_ledger > gpurun_out/bench_verify22_file_new$k.json 2> gpurun_out/bench_verify22_file_new$k.err || exit $?
rm -rf /tmp/upow_bench_ledger
UPOW_SQLITE_CACHE_MB=2 UPOW_WAL_AUTOCHECKPOINT=1000 timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 2 --ledger /tmp/upow_bench_ledger > gpurun_out/bench_verify22_file_old$k.json 2> gpurun_out/bench_verify22_file_old$k.err || exit $?
rm -rf /tmp/upow_bench_ledger
done
