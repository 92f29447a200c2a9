set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_p256.py -m gpu -x -q > gpurun_out/pytest_p256.log 2>&1; echo "p256 tests rc=$?"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o /tmp/ubench_valu && timeout -k 10 120 /tmp/ubench_valu > gpurun_out/ubench_valu.log 2>&1; echo "ubench rc=$?"
timeout -k 10 300 python scripts/p256_throughput.py > gpurun_out/p256_tp.log 2>&1; echo "tp rc=$?"
