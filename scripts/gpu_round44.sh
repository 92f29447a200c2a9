set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r44_pytest.log 2>&1 && echo pytest-ok &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r44_smoke.log 2>&1 && echo smoke-ok &&
timeout -k 10 300 python bench.py > gpurun_out/r44_bench.json 2> gpurun_out/r44_bench.err && cat gpurun_out/r44_bench.json &&
timeout -k 10 600 python bench.py --mode verify > gpurun_out/r44_verify.json 2> gpurun_out/r44_verify.err && cat gpurun_out/r44_verify.json &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof44 -o pow --output-format csv -- python3 bench.py --steps 5 --warmup 1 > gpurun_out/prof44.log 2>&1 && echo prof-ok
