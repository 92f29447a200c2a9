set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/pow_variants.py 0,1 > gpurun_out/variants2.log 2>&1 || exit 3
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/prof2 -o pmc --output-format csv -- python3 bench.py --steps 2 --warmup 0 --nonces 1073741824 > gpurun_out/prof2.log 2>&1 || exit 4
echo done
