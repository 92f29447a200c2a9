set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/p256_throughput.py > gpurun_out/p256_28.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof28 -o p256 --output-format csv -- python3 scripts/p256_throughput.py > gpurun_out/prof28.log 2>&1; echo "prof rc=$?"
