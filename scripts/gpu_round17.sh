set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
UPOW_TXCODEC_PROFILE=1 timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 1 > gpurun_out/bench_verify17.json 2> gpurun_out/bench_verify17.err || exit $?
