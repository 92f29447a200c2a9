set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python scripts/node_soak.py --rate 800 --seconds 30 --fanout1 120 --fanout2 200 --threads 16 --out gpurun_out/soak32.json > gpurun_out/soak32.log 2>&1; echo "soak rc=$?"
rm -rf gpurun_out/soak*/ledger.sqlite3*
