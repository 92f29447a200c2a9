set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_p256.py -m gpu -x -q > gpurun_out/pytest_p256_10.log 2>&1; rc=$?; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/p256_throughput.py > gpurun_out/p256_tp10.log 2>&1; echo "tp rc=$?"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc10 -o p256 --output-format csv -- python3 scripts/p256_throughput.py > gpurun_out/pmc10.log 2>&1; echo "pmc rc=$?"
