set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python scripts/node_soak.py --rate 1200 --seconds 30 --fanout1 180 --fanout2 200 --threads 8 --procs 4 --out gpurun_out/soak35.json > gpurun_out/soak35.log 2>&1; echo "soak rc=$?"
rm -rf gpurun_out/soak*/ledger.sqlite3* gpurun_out/soak*/push_*
