set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/p256_throughput.py > gpurun_out/p256_tp11.log 2>&1; echo "tp rc=$?"
