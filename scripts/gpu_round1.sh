set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "start $(date)"; rocm-smi --showproductname 2>&1 | head -20 > gpurun_out/smi.txt || true
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?"
timeout -k 10 240 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_v0.log 2>&1 || exit 3
echo "bench v0 done"
UPOW_POW_VARIANT=1 timeout -k 10 240 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_v1.log 2>&1 || exit 4
echo "bench v1 done"
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || exit 5
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 > gpurun_out/prof1.log 2>&1 || exit 6
echo "all done $(date)"
