# One parametrised GPU validation runner (replaces the per-lease gpu_roundN.sh scripts).
#
#   gpurun --timeout 1200 -- 'bash scripts/gpu_run.sh TAG [STEPS...]'
#
# STEPS (default: test smoke mine verify prof): any of
#   test     pytest -m gpu (one process, per-test thread timeout)
#   smoke    __graft_entry__.smoke()
#   mine     bench.py (driver default: PoW MH/s + verify side metrics)
#   verify   bench.py --mode verify --ledger <tmp dir> (file ledger, metric 2)
#   verifypool bench.py --mode verify --keys pool256 (file ledger, 256-key pool: the cache-friendly variant)
#   verifygrp bench.py --mode verify --grouped-txs 10% (grouped-signature txs on the native path)
#   verifymem bench.py --mode verify (in-memory ledger)
#   verifygov bench.py --mode verify --governance (file ledger; 12 inodes, 200 validators, 5,000 delegates)
#   verifygov5 bench.py --mode verify --governance-txs 5% (file ledger; 5 % of every block's txs are governance txs)
#   verifyaged bench.py --mode verify on a ledger aged to 2.5 M txs / 5 M UTXOs (20 blocks, SQL catch-up timed)
#   syncaged   bench.py --mode sync: 1,000 blocks replayed into the aged ledger
#   verifyaged60 60 blocks on the aged ledger (writer lag after every block, final drain)
#   aged:NAME:K=V,...  the same 60-block aged run with extra environment variables
#   cluster  forced single-rank RCCL cluster node, one chain (bench.py --mode verify under torchrun)
#   launch   bench.py --gpus 1 under torchrun (the driver's multi-rank entry form)
#   sync     bench.py --mode sync (chain-sync replay of a /get_blocks page, decode-ahead pipeline)
#   coloc    scripts/colocated.py (node + miner sharing the GPU)
#   prof     rocprofv3 --kernel-trace --stats over a short bench.py
#   vprof    rocprofv3 --kernel-trace --stats over the verify bench
#   tprof    rocprofv3 kernel + roctx marker trace of the verify bench, summarised by scripts/block_trace.py
#   tprofgov the same with 5 % governance txs per block
#   sprof    the same for the sync bench (200-tx blocks)
#   soak3    three node soaks at 1,200 tx/s (scripts/node_soak.py)
#   soak3pin the same, node pinned to CPUs 0-11 and miner + clients to 12-15 (inside the cgroup quota)
#   soakenv:NAME:K=V,...  one pinned soak with extra environment variables
#   verifyaged90 90 blocks on the aged ledger
#   verifyaged250 250 blocks on the aged ledger, across the retargets at blocks 100 and 200
#   p256ab   verify latency quad vs oct kernel: wall time, rocprofv3 kernel trace, SQ counters
#   p256n    kernel trace of quad vs oct at 1,024 / 4,096 / 8,192 / 8,300 signatures
#   soakc1   cluster node + DP miner under torchrun, forced single-rank RCCL, 40 tx/s (node_soak.py --cluster 1)
#   soakc1k  the same at 1,200 tx/s
#   verifyenv:NAME:K=V,...  verify bench (median of 3 segments) with extra environment variables
#   soakc3pin  three pinned cluster soaks alternating with three pinned plain soaks (1,200 tx/s)
#   clustersync  page-batched sync on a forced single-rank RCCL cluster vs plain, two interleaved pairs
#   leanshard:N  the N-rank lean node with the page plan's key stage sharded (default) vs replicated (UPOW_SHARD_KEYS=0)
#   sprofpage  rocprofv3 kernel trace + stats of the page-batched sync (200-tx blocks)
#   p256ab:VARIANT  P-256 kernels: the default build vs build-ab/native-VARIANT (latency, throughput, trace, counters)
#   isarates  issue cost of v_mad_u64_u32 / carry adds / 64-bit adds / f64 FMA / field products (scripts/isa_rates.hip)
#   collat   collective latencies over RCCL (scripts/collective_latency.py, forced single rank)
#   syncprof cProfile of the timed page sync of 0-20-tx blocks
#   bench:NAME:--a,1,...  bench.py with extra arguments (output bench_NAME.json)
#   py:<script.py>  any extra python script under scripts/ (args after a comma: py:x.py,--a,1)
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${1:-run}
shift || true
STEPS=${*:-test smoke mine verify prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for s in $STEPS; do
  echo "== $TAG: $s ($(date +%T))"
  case $s in
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
      tail -3 "$OUT/pytest.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
        || { cat "$OUT/smoke.log"; exit 1; }
      tail -1 "$OUT/smoke.log" ;;
    mine)
      timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" \
        || { tail -20 "$OUT/bench.err"; exit 1; }
      cat "$OUT/bench.json" ;;
    verify)
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 600 python bench.py --mode verify --ledger /tmp/upow_bench_ledger \
        > "$OUT/verify_file.json" 2> "$OUT/verify_file.err" || { tail -20 "$OUT/verify_file.err"; exit 1; }
      cat "$OUT/verify_file.json" | tee -a "$OUT/verify_runs.jsonl" | cut -c1-300 ;;
    verifypool)
      # the cache-friendly variant: a 256-key pool signs every tx and owns every output
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 600 python bench.py --mode verify --ledger /tmp/upow_bench_ledger --keys pool256 \
        > "$OUT/verify_pool256.json" 2> "$OUT/verify_pool256.err" || { tail -20 "$OUT/verify_pool256.err"; exit 1; }
      cat "$OUT/verify_pool256.json" ;;
    verifygrp)
      # 10 % of every block's txs with grouped signatures (4 inputs of two keys, 2 signatures)
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 600 python bench.py --mode verify --ledger /tmp/upow_bench_ledger --grouped-txs 10% \
        > "$OUT/verify_grouped10.json" 2> "$OUT/verify_grouped10.err" || { tail -20 "$OUT/verify_grouped10.err"; exit 1; }
      cat "$OUT/verify_grouped10.json" ;;
    verifygov5)
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 600 python bench.py --mode verify --ledger /tmp/upow_bench_ledger --governance-txs 5% \
        > "$OUT/verify_gov5.json" 2> "$OUT/verify_gov5.err" || { tail -20 "$OUT/verify_gov5.err"; exit 1; }
      cat "$OUT/verify_gov5.json" | tee -a "$OUT/verify_runs.jsonl" | cut -c1-300 ;;
    verifyaged)
      # chain scale: the ledger first aged to 2.5 M tx rows / 5 M UTXO rows, then 2 MB blocks incl. SQL catch-up
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 900 python -u bench.py --mode verify --ledger /tmp/upow_bench_ledger --age-txs 2500000 \
        --steps 20 --warmup 2 > "$OUT/verify_aged.json" 2> "$OUT/verify_aged.err" \
        || { tail -20 "$OUT/verify_aged.err"; exit 1; }
      cat "$OUT/verify_aged.json" ;;
    verifyaged60)
      # the aged ledger, default split, 60 blocks (the A of verifyaged8)
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 900 python -u bench.py --mode verify --ledger /tmp/upow_bench_ledger \
        --age-txs 2500000 --steps 60 --warmup 2 > "$OUT/verify_aged60.json" 2> "$OUT/verify_aged60.err" \
        || { tail -20 "$OUT/verify_aged60.err"; exit 1; }
      cat "$OUT/verify_aged60.json" | cut -c1-400 ;;
    aged:*)
      # aged:NAME:K=V,K=V  the 60-block aged-ledger run with extra environment (A/B of writer settings)
      spec=${s#aged:}; name=${spec%%:*}; envs=${spec#*:}
      rm -rf /tmp/upow_bench_ledger
      env ${envs//,/ } timeout -k 10 900 python -u bench.py --mode verify --ledger /tmp/upow_bench_ledger \
        --age-txs 2500000 --steps 60 --warmup 2 > "$OUT/verify_aged_$name.json" 2> "$OUT/verify_aged_$name.err" \
        || { tail -20 "$OUT/verify_aged_$name.err"; exit 1; }
      cut -c1-300 "$OUT/verify_aged_$name.json" ;;
    syncaged)
      # a 1,000-block sync (200 txs each) into the aged ledger, decode-ahead pipeline
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 900 python -u bench.py --mode sync --ledger /tmp/upow_bench_ledger --age-txs 2500000 \
        --steps 1000 --warmup 5 --txs 200 > "$OUT/sync_aged.json" 2> "$OUT/sync_aged.err" \
        || { tail -20 "$OUT/sync_aged.err"; exit 1; }
      cat "$OUT/sync_aged.json" ;;
    verifygov)
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 600 python bench.py --mode verify --ledger /tmp/upow_bench_ledger --governance \
        > "$OUT/verify_gov.json" 2> "$OUT/verify_gov.err" || { tail -20 "$OUT/verify_gov.err"; exit 1; }
      cat "$OUT/verify_gov.json" ;;
    sync)
      timeout -k 10 600 python bench.py --mode sync > "$OUT/sync.json" 2> "$OUT/sync.err" \
        || { tail -20 "$OUT/sync.err"; exit 1; }
      cat "$OUT/sync.json" ;;
    cluster)
      # one chain on a cluster node through the RCCL path, forced single rank (the 1-GPU box)
      rm -rf /tmp/upow_bench_ledger
      UPOW_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --mode verify --ledger /tmp/upow_bench_ledger \
        > "$OUT/verify_cluster.json" 2> "$OUT/verify_cluster.err" || { tail -20 "$OUT/verify_cluster.err"; exit 1; }
      grep '^{' "$OUT/verify_cluster.json" ;;
    launch)
      # the driver's plain command with an explicit --gpus 1 (no launcher hop) and the torchrun form
      timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29534 bench.py --gpus 1 --steps 5 --warmup 1 --verify-steps 2 \
        > "$OUT/bench_torchrun1.json" 2> "$OUT/bench_torchrun1.err" || { tail -20 "$OUT/bench_torchrun1.err"; exit 1; }
      grep '^{' "$OUT/bench_torchrun1.json" ;;
    coloc)
      timeout -k 10 300 python scripts/colocated.py --dispatch-log2 24 --prio high --out "$OUT/coloc.json" \
        > "$OUT/coloc.log" 2>&1 || { tail -20 "$OUT/coloc.log"; exit 1; }
      cat "$OUT/coloc.json" ;;
    verifymem)
      timeout -k 10 600 python bench.py --mode verify > "$OUT/verify_mem.json" 2> "$OUT/verify_mem.err" \
        || { tail -20 "$OUT/verify_mem.err"; exit 1; }
      cat "$OUT/verify_mem.json" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o pow --output-format csv \
        -- python3 bench.py --steps 5 --warmup 1 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
      echo prof-ok ;;
    powpmc)
      # counters of the PoW search kernel (one pass per counter group; the mining bench only): VALU
      # instructions per wave and per nonce, wave cycles, busy cycles, VALU-active cycles, GPU clock
      for grp in "SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" \
                 "SQ_INST_CYCLES_VALU SQ_INSTS_LDS"; do
        tag=$(echo "$grp" | cut -d' ' -f1 | tr 'A-Z' 'a-z')
        timeout -s KILL 120 rocprofv3 --pmc $grp -d "$OUT/powpmc_$tag" -o pow --output-format csv \
          -- python3 bench.py --steps 2 --warmup 1 --verify-steps 0 --sync-steps 0 > "$OUT/powpmc_$tag.log" 2>&1 \
          || { tail -20 "$OUT/powpmc_$tag.log"; exit 1; }
        find "$OUT/powpmc_$tag" -name '*counter_collection.csv' | head -1 | xargs -r grep -m 12 -E 'pow_search_kernel|Counter_Name' | cut -c1-400
      done ;;
    vprof)
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/vprof" -o verify --output-format csv \
        -- python3 bench.py --mode verify --ledger /tmp/upow_bench_ledger --steps 3 --warmup 1 \
        > "$OUT/vprof.log" 2>&1 || { tail -20 "$OUT/vprof.log"; exit 1; }
      echo vprof-ok ;;
    tprof)
      # one timeline: host stages (roctx ranges) + GPU kernels of the verify bench on a file ledger
      rm -rf /tmp/upow_bench_ledger
      UPOW_ROCTX=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -d "$OUT/tprof" -o verify \
        --output-format csv -- python3 bench.py --mode verify --ledger /tmp/upow_bench_ledger --steps 8 --warmup 2 \
        > "$OUT/tprof.log" 2>&1 || { tail -20 "$OUT/tprof.log"; exit 1; }
      python scripts/block_trace.py "$OUT/tprof" --out "$OUT/block_trace.json" | head -60 ;;
    tprofgov)
      # the same timeline with 5 % governance txs per block (stage-by-stage cost of the governance rules)
      rm -rf /tmp/upow_bench_ledger
      UPOW_ROCTX=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -d "$OUT/tprofgov" -o verify \
        --output-format csv -- python3 bench.py --mode verify --ledger /tmp/upow_bench_ledger --steps 8 --warmup 2 \
        --governance-txs 5% > "$OUT/tprofgov.log" 2>&1 || { tail -20 "$OUT/tprofgov.log"; exit 1; }
      python scripts/block_trace.py "$OUT/tprofgov" --out "$OUT/block_trace_gov.json" | head -60 ;;
    sprof)
      # the same timeline for the chain-sync replay (200-tx blocks through the decode-ahead pipeline)
      rm -rf /tmp/upow_bench_ledger
      UPOW_ROCTX=1 timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -d "$OUT/sprof" -o sync \
        --output-format csv -- python3 bench.py --mode sync --ledger /tmp/upow_bench_ledger --steps 300 --warmup 5 \
        --txs 200 > "$OUT/sprof.log" 2>&1 || { tail -20 "$OUT/sprof.log"; exit 1; }
      python scripts/block_trace.py "$OUT/sprof" --out "$OUT/sync_trace.json" | head -80 ;;
    soakc1)
      # BASELINE config 5 launcher on the 1-GPU box: cluster node + DP miner under torchrun, forced
      # single-rank RCCL (scripts/node_soak.py --cluster 1)
      timeout -k 10 420 python -u scripts/node_soak.py --cluster 1 --rate 40 --seconds 45 --difficulty 9 \
        --out "$OUT/soak_cluster1.json" > "$OUT/soak_cluster1.log" 2>&1 || { tail -30 "$OUT/soak_cluster1.log"; exit 1; }
      tail -1 "$OUT/soak_cluster1.log" | cut -c1-900 ;;
    soakc1k)
      # the same at 1,200 tx/s
      timeout -k 10 420 python -u scripts/node_soak.py --cluster 1 --rate 1200 --seconds 45 --difficulty 9 --procs 4 \
        --threads 8 --fanout1 255 --fanout2 220 --out "$OUT/soak_cluster1_1200.json" > "$OUT/soak_cluster1_1200.log" 2>&1 \
        || { tail -30 "$OUT/soak_cluster1_1200.log"; exit 1; }
      tail -1 "$OUT/soak_cluster1_1200.log" | cut -c1-900 ;;
    verifyenv:*)
      # verifyenv:NAME:K=V,K=V  the verify bench (file ledger, median of 3 segments of 10 blocks) with extra env
      spec=${s#verifyenv:}; name=${spec%%:*}; envs=${spec#*:}
      rm -rf /tmp/upow_bench_ledger
      env ${envs//,/ } timeout -k 10 600 python -u bench.py --mode verify --ledger /tmp/upow_bench_ledger --segments 3 \
        > "$OUT/verifyenv_$name.json" 2> "$OUT/verifyenv_$name.err" || { tail -20 "$OUT/verifyenv_$name.err"; exit 1; }
      cut -c1-400 "$OUT/verifyenv_$name.json" ;;
    soakc3pin)
      # three cluster soaks (forced single-rank RCCL node + DP miner) with the r4e placement: node on CPUs 0-11,
      # miner and pushing clients on 12-15 (inside the cgroup quota), alternating with three plain pinned soaks
      for i in 1 2 3; do
        UPOW_CPU_AFFINITY=0-11 timeout -k 10 420 python -u scripts/node_soak.py --cluster 1 --rate 1200 --seconds 45 \
          --difficulty 9 --procs 4 --threads 8 --fanout1 255 --fanout2 220 --client-cpus 12-15 \
          --out "$OUT/soakc_pin_$i.json" > "$OUT/soakc_pin_$i.log" 2>&1 || { tail -30 "$OUT/soakc_pin_$i.log"; exit 1; }
        tail -1 "$OUT/soakc_pin_$i.log" | cut -c1-400
        UPOW_CPU_AFFINITY=0-11 timeout -k 10 420 python -u scripts/node_soak.py --rate 1200 --seconds 45 --difficulty 9 \
          --procs 4 --threads 8 --fanout1 255 --fanout2 220 --client-cpus 12-15 --out "$OUT/soakp_pin_$i.json" \
          > "$OUT/soakp_pin_$i.log" 2>&1 || { tail -30 "$OUT/soakp_pin_$i.log"; exit 1; }
        tail -1 "$OUT/soakp_pin_$i.log" | cut -c1-400
      done ;;
    p256ab)
      # single-block verify latency, quad (4 lanes/signature) vs oct (8 lanes/signature): wall time, kernel
      # trace, and SQ counters for each kernel (own rocprofv3 pass, no other trace domains)
      timeout -k 10 300 python -u scripts/p256_latency.py 4:64,8:64 > "$OUT/p256_latency.txt" 2>&1 \
        || { tail -20 "$OUT/p256_latency.txt"; exit 1; }
      tail -1 "$OUT/p256_latency.txt"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/p256kt" -o p256 --output-format csv \
        -- python3 scripts/p256_latency.py 4:64,8:64 > "$OUT/p256kt.log" 2>&1 || { tail -20 "$OUT/p256kt.log"; exit 1; }
      timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU -d "$OUT/p256pmc" -o pmc --output-format csv \
        -- python3 scripts/p256_latency.py 4:64,8:64 > "$OUT/p256pmc.log" 2>&1 || { tail -20 "$OUT/p256pmc.log"; exit 1; }
      echo p256ab-ok ;;
    p256n)
      # quad vs oct kernel time against the signature count (waves per SIMD: n/16 vs n/8 waves on 1,024 SIMDs)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/p256n" -o p256n --output-format csv \
        -- python3 scripts/p256_latency.py 4:64:1024,8:64:1024,4:64:4096,8:64:4096,4:64:8192,8:64:8192,4:64,8:64 \
        > "$OUT/p256n.log" 2>&1 || { tail -20 "$OUT/p256n.log"; exit 1; }
      tail -1 "$OUT/p256n.log" ;;
    soak3pin)
      # the same three soaks with the job pinned inside the cgroup's CPU quota: node on CPUs 0-11, miner and
      # pushing clients on 12-15 (a burst over the quota's width throttles every thread of the node)
      for i in 1 2 3; do
        UPOW_CPU_AFFINITY=0-11 timeout -k 10 420 python -u scripts/node_soak.py --rate 1200 --seconds 45 --difficulty 9 \
          --procs 4 --threads 8 --fanout1 255 --fanout2 220 --client-cpus 12-15 --out "$OUT/soakpin_$i.json" \
          > "$OUT/soakpin_$i.log" 2>&1 || { tail -30 "$OUT/soakpin_$i.log"; exit 1; }
        tail -1 "$OUT/soakpin_$i.log" | cut -c1-600
      done ;;
    soakenv:*)
      # soakenv:NAME:K=V,K=V  one pinned 1,200 tx/s soak with extra environment (A/B of node settings)
      spec=${s#soakenv:}; name=${spec%%:*}; envs=${spec#*:}
      env ${envs//,/ } UPOW_CPU_AFFINITY=0-11 timeout -k 10 420 python -u scripts/node_soak.py --rate 1200 --seconds 45 \
        --difficulty 9 --procs 4 --threads 8 --fanout1 255 --fanout2 220 --client-cpus 12-15 \
        --out "$OUT/soakenv_$name.json" > "$OUT/soakenv_$name.log" 2>&1 || { tail -30 "$OUT/soakenv_$name.log"; exit 1; }
      tail -1 "$OUT/soakenv_$name.log" | cut -c1-400 ;;
    verifyaged90)
      # the aged ledger, 90 blocks (the pre-mined headers keep the start difficulty below block 100): backlog over a long run
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 900 python -u bench.py --mode verify --ledger /tmp/upow_bench_ledger \
        --age-txs 2500000 --steps 90 --warmup 2 > "$OUT/verify_aged90.json" 2> "$OUT/verify_aged90.err" \
        || { tail -20 "$OUT/verify_aged90.err"; exit 1; }
      cut -c1-400 "$OUT/verify_aged90.json" ;;
    verifyaged250)
      # the aged ledger, 250 blocks: the headers are mined at the difficulty the chain computes, so the run
      # crosses the retargets at blocks 100 and 200 on the native path
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 1000 python -u bench.py --mode verify --ledger /tmp/upow_bench_ledger \
        --age-txs 2500000 --steps 250 --warmup 2 > "$OUT/verify_aged250.json" 2> "$OUT/verify_aged250.err" \
        || { tail -20 "$OUT/verify_aged250.err"; exit 1; }
      cut -c1-600 "$OUT/verify_aged250.json" ;;
    soak3)
      # three consecutive node soaks at 1,200 tx/s (node + GPU miner CLI + 4 x 8 pushing clients)
      for i in 1 2 3; do
        timeout -k 10 420 python -u scripts/node_soak.py --rate 1200 --seconds 45 --difficulty 9 --procs 4 --threads 8 \
          --fanout1 255 --fanout2 220 --out "$OUT/soak_$i.json" > "$OUT/soak_$i.log" 2>&1 \
          || { tail -30 "$OUT/soak_$i.log"; exit 1; }
        tail -1 "$OUT/soak_$i.log" | cut -c1-600
      done ;;
    clustersync)
      # page-batched sync of one chain on a forced single-rank RCCL cluster node vs the plain node (three
      # interleaved A/B pairs)
      for k in 1 2 3; do
        rm -rf /tmp/upow_bench_ledger
        UPOW_FORCE_DIST=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
          --master-addr 127.0.0.1 --master-port 2954$k bench.py --gpus 1 --mode sync --txs 200 --steps 1000 --warmup 5 \
          --ledger /tmp/upow_bench_ledger > "$OUT/sync_cluster_$k.json" 2> "$OUT/sync_cluster_$k.err" \
          || { tail -20 "$OUT/sync_cluster_$k.err"; exit 1; }
        grep '^{' "$OUT/sync_cluster_$k.json" | cut -c1-300
        rm -rf /tmp/upow_bench_ledger
        timeout -k 10 600 python bench.py --mode sync --txs 200 --steps 1000 --warmup 5 --ledger /tmp/upow_bench_ledger \
          > "$OUT/sync_plain_$k.json" 2> "$OUT/sync_plain_$k.err" || { tail -20 "$OUT/sync_plain_$k.err"; exit 1; }
        cut -c1-300 "$OUT/sync_plain_$k.json"
      done ;;
    leansync:*)
      # page-batched sync of one chain on an N-rank cluster node sharing this one GPU (host collectives:
      # UPOW_DIST_BACKEND=gloo; every rank's P-256, UTXO and decompression work on the GPU), lean followers
      # (default) vs full followers (UPOW_CLUSTER_LEAN=0): per-rank host CPU per block
      N=${s#leansync:}
      for mode in 1 0; do
        rm -rf /tmp/upow_bench_ledger
        UPOW_CLUSTER_LEAN=$mode UPOW_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port 2957$mode bench.py --gpus "$N" --mode sync \
          --txs 200 --steps 1000 --warmup 5 --ledger /tmp/upow_bench_ledger > "$OUT/leansync_${N}_lean$mode.json" \
          2> "$OUT/leansync_${N}_lean$mode.err" || { tail -20 "$OUT/leansync_${N}_lean$mode.err"; exit 1; }
        grep '^{' "$OUT/leansync_${N}_lean$mode.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('world','value','ms_per_step','blocks_per_s','rank_cpu_ms_per_block','rank_cpu_ms_per_block_ex_p256','follower_cpu_vs_leader','lean_followers')})"
      done ;;
    leanshard:*)
      # the same N-rank lean node with the page plan's key stage sharded over the ranks (default) vs replicated
      # on every rank (UPOW_SHARD_KEYS=0)
      N=${s#leanshard:}
      for mode in 1 0; do
        rm -rf /tmp/upow_bench_ledger
        UPOW_SHARD_KEYS=$mode UPOW_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node "$N" --master-addr 127.0.0.1 --master-port 2958$mode bench.py --gpus "$N" --mode sync \
          --txs 200 --steps 1000 --warmup 5 --ledger /tmp/upow_bench_ledger > "$OUT/leanshard_${N}_shard$mode.json" \
          2> "$OUT/leanshard_${N}_shard$mode.err" || { tail -20 "$OUT/leanshard_${N}_shard$mode.err"; exit 1; }
        grep '^{' "$OUT/leanshard_${N}_shard$mode.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ('world','value','ms_per_step','blocks_per_s','rank_cpu_ms_per_block','rank_cpu_ms_per_block_ex_p256','follower_cpu_vs_leader','lean_followers')})"
      done ;;
    sprofpage)
      # rocprofv3 kernel trace of the page-batched sync (200-tx blocks)
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/sprofpage" -o sync --output-format csv \
        -- python3 bench.py --mode sync \
        --txs 200 --steps 1000 --warmup 5 --ledger /tmp/upow_bench_ledger > "$OUT/sprofpage.json" 2> "$OUT/sprofpage.err" \
        || { tail -20 "$OUT/sprofpage.err"; exit 1; }
      find "$OUT/sprofpage" -name '*kernel_stats.csv' | head -1 | xargs -r head -25 ;;
    collat)
      # latency of the cluster collectives over RCCL (forced single-rank group on the one GPU)
      UPOW_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29561 scripts/collective_latency.py > "$OUT/collat.json" \
        2> "$OUT/collat.err" || { tail -20 "$OUT/collat.err"; exit 1; }
      grep '^{' "$OUT/collat.json" ;;
    syncprof)
      # cProfile of the timed page-batched sync of mainnet-shaped blocks (0-20 txs)
      rm -rf /tmp/upow_bench_ledger
      UPOW_BENCH_PROFILE="$OUT/syncprof.txt" timeout -k 10 600 python bench.py --mode sync --txs-range 0-20 \
        --steps 2000 --warmup 5 --ledger /tmp/upow_bench_ledger > "$OUT/syncprof.json" 2> "$OUT/syncprof.err" \
        || { tail -20 "$OUT/syncprof.err"; exit 1; }
      cut -c1-300 "$OUT/syncprof.json" ;;
    p256ab:*)
      # p256ab:VARIANT  A/B of the P-256 kernels: the build default ("cur") against an A/B build
      # (build-ab/native-VARIANT, upow_amd/_build.py AB_VARIANTS): block latency, batch throughput, kernel
      # trace, SQ counters (own rocprofv3 pass, no other trace domains)
      var=${s#p256ab:}
      ALT=$(ls build-ab/native-$var/_native*.so)
      for v in cur $var; do
        SO=""; [ $v = $var ] && SO=$ALT
        UPOW_NATIVE_SO=$SO timeout -k 10 300 python -u scripts/p256_latency.py 4:64,8:64 > "$OUT/p256lat_$v.txt" 2>&1 \
          || { tail -20 "$OUT/p256lat_$v.txt"; exit 1; }
        echo "$v latency $(tail -1 "$OUT/p256lat_$v.txt")"
        UPOW_NATIVE_SO=$SO timeout -k 10 300 python -u scripts/p256_throughput.py > "$OUT/p256thr_$v.txt" 2>&1 \
          || { tail -20 "$OUT/p256thr_$v.txt"; exit 1; }
        echo "$v throughput $(tail -1 "$OUT/p256thr_$v.txt")"
        UPOW_NATIVE_SO=$SO timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/p256kt_$v" -o p256 \
          --output-format csv -- python3 scripts/p256_latency.py 4:64,8:64 > "$OUT/p256kt_$v.log" 2>&1 \
          || { tail -20 "$OUT/p256kt_$v.log"; exit 1; }
        UPOW_NATIVE_SO=$SO timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
          SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_SALU -d "$OUT/p256pmc_$v" -o pmc \
          --output-format csv -- python3 scripts/p256_latency.py 4:64,8:64 > "$OUT/p256pmc_$v.log" 2>&1 \
          || { tail -20 "$OUT/p256pmc_$v.log"; exit 1; }
      done
      echo p256ab-ok ;;
    isarates)
      # issue cost of the candidate big-integer instructions (scripts/isa_rates.hip, built into build-ab/)
      timeout -k 10 120 ./build-ab/isa_rates > "$OUT/isa_rates.json" 2>&1 || { cat "$OUT/isa_rates.json"; exit 1; }
      cat "$OUT/isa_rates.json" ;;
    bench:*)
      # bench:NAME:--arg,value,...  one bench.py run with extra arguments (file ledger under /tmp)
      spec=${s#bench:}; name=${spec%%:*}; rest=${spec#*:}; rest=${rest//,/ }
      rm -rf /tmp/upow_bench_ledger
      timeout -k 10 900 python -u bench.py $rest > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
        || { tail -30 "$OUT/bench_$name.err"; exit 1; }
      cut -c1-600 "$OUT/bench_$name.json" ;;
    py:*)
      spec=${s#py:}; script=${spec%%,*}; rest=""
      [ "$spec" != "$script" ] && rest=${spec#*,} && rest=${rest//,/ }
      timeout -k 10 600 python -u "scripts/$script" $rest > "$OUT/${script%.py}.out" 2>&1 \
        || { tail -30 "$OUT/${script%.py}.out"; exit 1; }
      tail -15 "$OUT/${script%.py}.out" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "== $TAG done"
