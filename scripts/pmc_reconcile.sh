# PoW VALU-count reconciliation (docs/PERF.md §1): SQ_INSTS_VALU / SQ_WAVES on a calibration kernel
# with a known instruction count (tools/ubench_valu c), then on the PoW bench, one rocprofv3 pass each.
#   gpurun -- 'bash scripts/pmc_reconcile.sh TAG'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_SALU -d "$OUT/calib" -o calib \
  --output-format csv -- ./tools/ubench_valu c > "$OUT/calib.log" 2>&1 || { tail -20 "$OUT/calib.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_INSTS_SALU -d "$OUT/pow" -o pow \
  --output-format csv -- python3 bench.py --steps 2 --warmup 0 --verify-steps 0 > "$OUT/pow.log" 2>&1 \
  || { tail -20 "$OUT/pow.log"; exit 1; }
echo pmc-ok
