set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for ns in 1 0; do
  UPOW_NATIVE_SQL=$ns timeout -k 10 400 python bench.py --mode verify --steps 3 --warmup 1 > gpurun_out/bench_verify15_ns$ns.json 2> gpurun_out/bench_verify15_ns$ns.err || exit $?
done
