set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_utxo.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r38_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r38_pytest.log; exit $rc
