set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python scripts/node_soak.py --rate 400 --seconds 40 --fanout1 80 --fanout2 200 --threads 8 --out gpurun_out/soak31.json > gpurun_out/soak31.log 2>&1; echo "soak rc=$?"
rm -rf gpurun_out/soak*/ledger.sqlite3*
