set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_p256.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_p256_24.log 2>&1 || exit $?
timeout -k 10 300 python scripts/p256_throughput.py > gpurun_out/p256_24.txt 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc24 -o p256 --output-format csv -- python3 scripts/p256_throughput.py > gpurun_out/pmc24.log 2>&1; echo "pmc rc=$?"
