set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python scripts/node_soak.py --rate 400 --seconds 40 --fanout1 80 --fanout2 200 --threads 8 --out gpurun_out/soak30.json > gpurun_out/soak30.log 2>&1; echo "soak rc=$?"
timeout -k 10 600 python bench.py --mode verify --steps 3 --warmup 1 --object-path > gpurun_out/bench_verify30_obj.json 2> gpurun_out/bench_verify30_obj.err || exit $?
rm -rf gpurun_out/soak*/ledger.sqlite3* 
