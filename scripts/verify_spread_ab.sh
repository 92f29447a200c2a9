# Verify side-metric spread A/B (docs/ROUND6.md §4): the verify bench (file ledger, 3 segments of 10 blocks)
# with a 2- or 10-block untimed warmup and the WAL checkpointer's period at 0.5 s (default) or 2 s, each
# variant twice, interleaved. Output: gpurun_out/$1/spread_<variant>_<k>.json
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-spread}
mkdir -p "$OUT"
export TMPDIR=/tmp
for k in 1 2; do
  for v in base w10 ck2 w10ck2; do
    case $v in
      base) W=2; P=0.5 ;; w10) W=10; P=0.5 ;; ck2) W=2; P=2 ;; w10ck2) W=10; P=2 ;;
    esac
    rm -rf /tmp/upow_bench_ledger
    UPOW_WAL_CHECKPOINT_PERIOD=$P timeout -k 10 300 python -u bench.py --mode verify --ledger /tmp/upow_bench_ledger \
      --segments 3 --steps 10 --warmup $W > "$OUT/spread_${v}_$k.json" 2> "$OUT/spread_${v}_$k.err" \
      || { tail -20 "$OUT/spread_${v}_$k.err"; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/spread_${v}_$k.json')); s=d['segments_tx_per_s']; print('$v $k', d['value'], s, round((max(s)-min(s))/d['value']*100,1), '%')"
  done
done
