set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pow.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_pow14.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/pow_variants.py 0,1,2 > gpurun_out/pow_variants14.txt 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/pmc14 -o lds --output-format csv -- python3 bench.py --steps 2 --warmup 0 --nonces 1073741824 --variant 2 > gpurun_out/pmc14.log 2>&1; echo "pmc rc=$?"
