set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
UPOW_SOAK_PROFILE=1 timeout -k 10 900 python scripts/node_soak.py --rate 800 --seconds 30 --fanout1 120 --fanout2 200 --threads 16 --out gpurun_out/soak34.json > gpurun_out/soak34.log 2>&1; echo "soak rc=$?"
for f in gpurun_out/soak*/node.prof; do python -c "import pstats,sys; pstats.Stats(sys.argv[1]).sort_stats('tottime').print_stats(45)" $f > gpurun_out/node_prof34_tottime.txt 2>&1; python -c "import pstats,sys; pstats.Stats(sys.argv[1]).sort_stats('cumulative').print_stats(60)" $f > gpurun_out/node_prof34_cum.txt 2>&1; done
rm -rf gpurun_out/soak*/ledger.sqlite3* gpurun_out/soak*/node.prof
