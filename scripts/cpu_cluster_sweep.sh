#!/usr/bin/env bash
# The cluster sync bench on the CPU (gloo, host P-256, host UTXO table): one bench.py --mode sync line per world
# size, written to <outdir>/w<N><tag>.json, plus a summary of blocks/s and per-rank CPU per block.
#
#   scripts/cpu_cluster_sweep.sh <outdir> [worlds="1 2 4 8"] [tag]     (extra env passes through, e.g.
#   UPOW_SHARD_KEYS=0 UPOW_CLUSTER_LEAN=0 for the A/B branches)
#
# World 1 is the plain node (no cluster). Sized for the 8-CPU build container: 100 blocks of 200 txs.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:?outdir}
WORLDS=${2:-"1 2 4 8"}
TAG=${3:-}
STEPS=${SWEEP_STEPS:-100}
mkdir -p "$OUT"
export UPOW_DISABLE_GPU=1 UPOW_LOG_LEVEL=WARNING
for w in $WORLDS; do
  f="$OUT/w${w}${TAG}.json"
  if [ "$w" = 1 ]; then
    timeout -k 10 900 python bench.py --mode sync --steps "$STEPS" --warmup 4 --txs 200 > "$f.log" 2>&1
  else
    port=$((29600 + RANDOM % 300))
    timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$w" --master-addr 127.0.0.1 \
      --master-port "$port" bench.py --mode sync --gpus "$w" --steps "$STEPS" --warmup 4 --txs 200 > "$f.log" 2>&1
  fi
  grep -E '^\{"metric"' "$f.log" | tail -1 > "$f"
done
python - "$OUT" "$TAG" <<'EOF'
import glob, json, os, sys
out, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(os.path.join(out, f'w*{tag}.json'))):
    try:
        d = json.load(open(f))
    except ValueError:
        print(os.path.basename(f), 'no result line'); continue
    keep = ('world', 'blocks_per_s', 'ms_per_step', 'rank_cpu_ms_per_block', 'rank_cpu_ms_per_block_ex_p256',
            'follower_cpu_vs_leader', 'lean_followers')
    src = d.get('sync', d)
    print(os.path.basename(f), {k: src.get(k, d.get(k)) for k in keep})
EOF
