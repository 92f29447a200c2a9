set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python scripts/sqlite_calib.py > gpurun_out/calib18.json 2>&1 || exit $?
for k in 1 2 3; do
  timeout -k 10 400 python bench.py --mode verify --steps 5 --warmup 1 > gpurun_out/bench_verify18_$k.json 2> gpurun_out/bench_verify18_$k.err || exit $?
done
