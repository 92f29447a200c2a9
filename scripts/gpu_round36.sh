set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r36_pytest.log 2>&1 && echo pytest-ok &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r36_smoke.log 2>&1 && echo smoke-ok &&
timeout -k 10 300 python bench.py > gpurun_out/r36_bench.json 2> gpurun_out/r36_bench.err && cat gpurun_out/r36_bench.json &&
timeout -k 10 600 python bench.py --mode verify > gpurun_out/r36_verify.json 2> gpurun_out/r36_verify.err && cat gpurun_out/r36_verify.json
