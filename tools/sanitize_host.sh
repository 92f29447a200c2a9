#!/usr/bin/env bash
# Host code under the sanitizers (CPU only: GPU sanitizers are not used on this pool).
#
#   tools/sanitize_host.sh [outdir]          (FUZZ_SECONDS=N per fuzz target, default 20)
#
# 1. tools/host_selftest.cpp + the host crypto (SHA-256, SHA-NI, base58, P-256) under ASan + UBSan;
#    the host worker pool (csrc/thread_pool.h) under ThreadSanitizer.
# 2. libFuzzer + ASan + UBSan on the parsers of untrusted network input: the tx decoder every pushed tx and
#    every peer block goes through (csrc/txdecode.h, tools/fuzz/fuzz_txdecode.cpp) and the HTTP/1.1 +
#    WebSocket framing of every request (csrc/http_wire.h, tools/fuzz/fuzz_http.cpp), seeded with valid
#    txs / requests / frames (tools/fuzz/make_corpus.py); and the span JSON parser of every /push_block body
#    and /get_blocks page (csrc/jsonspan.cpp, tools/fuzz/fuzz_jsonspan.cpp: an embedded interpreter, every
#    accepted input checked against json.loads), seeded with the committed corpus tools/fuzz/corpus/jsonspan
#    plus generated bodies, run for FUZZ_JSONSPAN_RUNS executions (default 10 M) over FUZZ_JOBS forked
#    workers. ASan's global redzones are off for these builds
#    (-mllvm -asan-globals=0): the fuzzer runtime and the target register some header-defined globals
#    twice, which ASan reports as an ODR violation before the first input.
# 3. The whole native extension built instrumented (python -m upow_amd._build --variant asan|tsan) and
#    loaded by an interpreter linked with the same runtime (tools/pysan.c, UPOW_NATIVE_SO): the Python
#    tests of every pybind11 module run under ASan + UBSan (txcodec, jsonspan, http_wire, mempool_index, utxo_host,
#    ledger_writer, gov_index, log_appender, the block path) and the threaded ones under TSan
#    (mempool index lookups racing a GIL-free confirm, the journal writer's I/O and materialiser threads,
#    the log appender's writer thread).
set -euo pipefail
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=${1:-build/sanitize}
FUZZ_SECONDS=${FUZZ_SECONDS:-20}
mkdir -p "$OUT"
SAN_HOST="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined"
CXX=/opt/rocm/llvm/bin/clang++
CFLAGS="-O1 -g -fno-omit-frame-pointer -std=c++17 -I/opt/rocm/include"
# HIP translation unit: device code at -O3 as in the build; host side instrumented, at -O0
# with line tables: the force-inlined 256-bit field code of the four-lane emulation takes ~10 minutes
# to optimise under ASan + UBSan instrumentation, ~1 minute unoptimised
stale() {  # $1 = object, rest = inputs: rebuild when any input is newer
  local o=$1; shift
  [ ! -f "$o" ] && return 0
  for i in "$@"; do [ "$i" -nt "$o" ] && return 0; done
  return 1
}
HDRS="csrc/native.h csrc/sha256_common.h csrc/p256_field.h csrc/p256_verify.h"
echo "== [1] host selftest (ASan + UBSan) and host pool (TSan)"
for h in p256 p256_batch; do  # the verify TU and the one-lane batch kernel's TU it launches
  if stale "$OUT/$h.o" csrc/$h.hip $HDRS; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Xarch_host -O0 -g1 -std=c++17 -I/opt/rocm/include $SAN_HOST \
      -c csrc/$h.hip -o "$OUT/$h.o"
  fi
done
for f in csrc/sha256_host.cpp csrc/sha256_ni.cpp csrc/base58.cpp csrc/p256_host.cpp tools/host_selftest.cpp; do
  o="$OUT/$(basename "${f%.cpp}").o"
  if stale "$o" "$f" $HDRS; then
    $CXX $CFLAGS -fsanitize=address,undefined -fno-sanitize-recover=undefined -pthread -c "$f" -o "$o"
  fi
done
$CXX -fsanitize=address,undefined -pthread "$OUT"/host_selftest.o "$OUT"/p256.o "$OUT"/p256_batch.o "$OUT"/sha256_host.o \
  "$OUT"/sha256_ni.o "$OUT"/base58.o "$OUT"/p256_host.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -o "$OUT/host_selftest"
# leak checking off: the HIP runtime keeps process-lifetime allocations
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/host_selftest"
# ThreadSanitizer on the host worker pool (csrc/thread_pool.h)
if stale "$OUT/pool_selftest" tools/pool_selftest.cpp csrc/thread_pool.h; then
  $CXX -O1 -g -std=c++17 -fsanitize=thread -pthread -Icsrc tools/pool_selftest.cpp -o "$OUT/pool_selftest"
fi
TSAN_OPTIONS=halt_on_error=1 "$OUT/pool_selftest"

echo "== [2] libFuzzer targets (ASan + UBSan), ${FUZZ_SECONDS} s each"
FZ="-O1 -g -fno-omit-frame-pointer -std=c++17 -fsanitize=fuzzer,address,undefined -fno-sanitize-recover=undefined -mllvm -asan-globals=0 -I/opt/rocm/include"
if stale "$OUT/fuzz_http" tools/fuzz/fuzz_http.cpp csrc/http_wire.h; then
  $CXX $FZ tools/fuzz/fuzz_http.cpp -o "$OUT/fuzz_http"
fi
if stale "$OUT/fuzz_txdecode" tools/fuzz/fuzz_txdecode.cpp csrc/txdecode.h csrc/base58.cpp csrc/sha256_host.cpp $HDRS; then
  $CXX $FZ tools/fuzz/fuzz_txdecode.cpp csrc/base58.cpp csrc/sha256_ni.cpp csrc/sha256_host.cpp -pthread -o "$OUT/fuzz_txdecode"
fi
PYINC=$(python3 -c 'import sysconfig; print(sysconfig.get_paths()["include"])')
PBINC=$(python3 -c 'import pybind11; print(pybind11.get_include())')
if stale "$OUT/fuzz_jsonspan" tools/fuzz/fuzz_jsonspan.cpp csrc/jsonspan.cpp; then
  $CXX $FZ -I"$PYINC" -I"$PBINC" tools/fuzz/fuzz_jsonspan.cpp -L/usr/lib/x86_64-linux-gnu -lpython3.10 -o "$OUT/fuzz_jsonspan"
fi
UPOW_NO_TORCH=1 python3 tools/fuzz/make_corpus.py "$OUT/corpus" > /dev/null
for t in http txdecode; do
  seeds=$OUT/corpus/${t#txdecode}; [ "$t" = txdecode ] && seeds=$OUT/corpus/tx
  mkdir -p "$OUT/work_$t"
  (cd "$OUT" && ./fuzz_$t -max_total_time="$FUZZ_SECONDS" -print_final_stats=1 "work_$t" "$ROOT/$seeds" > "fuzz_$t.log" 2>&1) \
    || { tail -40 "$OUT/fuzz_$t.log"; exit 1; }
  echo "fuzz $t: $(grep -E '^Done [0-9]+ runs' "$OUT/fuzz_$t.log") (corpus $(ls "$OUT/work_$t" | wc -l) inputs, no crash)"
done
# the span parser: a run-count target over forked workers (each execution calls into the interpreter, ~5 k/s
# per worker); the committed corpus grows by what this run finds (merged, minimised: -merge=1)
RUNS=${FUZZ_JSONSPAN_RUNS:-10000000}
JOBS=${FUZZ_JOBS:-8}
mkdir -p "$OUT/work_jsonspan"
(cd "$OUT" && PYTHONMALLOC=malloc ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
  ./fuzz_jsonspan -fork="$JOBS" -runs="$RUNS" -ignore_crashes=0 -print_final_stats=1 work_jsonspan \
  "$ROOT/tools/fuzz/corpus/jsonspan" "$ROOT/$OUT/corpus/json" > fuzz_jsonspan.log 2>&1) \
  || { tail -40 "$OUT/fuzz_jsonspan.log"; exit 1; }
echo "fuzz jsonspan: $(grep -cE '^#[0-9]+: cov' "$OUT/fuzz_jsonspan.log") fork rounds, $(grep -oE 'exec/s: [0-9]+' "$OUT/fuzz_jsonspan.log" | tail -1), no crash, no json.loads difference"
if [ -n "${FUZZ_MERGE:-}" ]; then  # fold what the run found into the committed corpus
  (cd "$OUT" && ./fuzz_jsonspan -merge=1 "$ROOT/tools/fuzz/corpus/jsonspan" work_jsonspan > fuzz_jsonspan_merge.log 2>&1)
fi

echo "== [3] the native extension instrumented, its Python tests under ASan + UBSan and TSan"
python3 -m upow_amd._build --variant asan -j 8 > /dev/null
python3 -m upow_amd._build --variant tsan -j 8 > /dev/null
PYINC=$(python3 -c 'import sysconfig; print(sysconfig.get_paths()["include"])')
for v in asan tsan; do
  san=$([ $v = asan ] && echo "-fsanitize=address,undefined" || echo "-fsanitize=thread")
  if stale "$OUT/pysan_$v" tools/pysan.c; then
    $CXX -x c++ -O1 -g $san -I"$PYINC" tools/pysan.c -L/usr/lib/x86_64-linux-gnu -lpython3.10 -Wl,--no-as-needed -lstdc++ \
      -o "$OUT/pysan_$v"
  fi
done
EXT=$(python3 -c 'import sysconfig; print(sysconfig.get_config_var("EXT_SUFFIX"))')
export UPOW_NO_TORCH=1 UPOW_DISABLE_GPU=1 PYTHONMALLOC=malloc
# three groups of test files in parallel processes (one ASan interpreter each; the files use ephemeral ports
# and their own temporary directories), so the stage takes the time of its slowest group
ASAN_GROUPS=("tests/test_utxo.py tests/test_txcodec.py tests/test_hexspans.py tests/test_http_server.py"
  "tests/test_fastpath.py tests/test_fastpath_governance.py tests/test_rollback_undo.py tests/test_gov_cascade.py"
  "tests/test_crash_recovery.py tests/test_ledger_writer.py tests/test_mempool_index.py tests/test_log_appender.py tests/test_process_tuning.py")
pids=()
for g in 0 1 2; do
  UPOW_NATIVE_SO=$ROOT/build/native-asan/_native$EXT ASAN_OPTIONS=detect_leaks=0:detect_odr_violation=0:abort_on_error=1 \
    UBSAN_OPTIONS=print_stacktrace=1 timeout -k 10 1500 "$OUT/pysan_asan" -m pytest -q -x -m "not gpu" -p no:cacheprovider \
    ${ASAN_GROUPS[$g]} > "$OUT/pytest_asan_$g.log" 2>&1 &
  pids+=($!)
done
asan_ok=1
for g in 0 1 2; do
  wait "${pids[$g]}" || { echo "ASan group $g failed:"; tail -60 "$OUT/pytest_asan_$g.log"; asan_ok=0; }
done
[ $asan_ok = 1 ] || exit 1
python3 - "$OUT" > "$OUT/pytest_asan.log" <<'PYEOF'
import re, sys
total = 0
for g in range(3):
    last = open(f'{sys.argv[1]}/pytest_asan_{g}.log').read().strip().splitlines()[-1]
    m = re.search(r'(\d+) passed', last)
    total += int(m.group(1)) if m else 0
    print(f'group {g}: {last}')
print(f'{total} passed in 3 parallel groups')
PYEOF
echo "python tests under ASan + UBSan: $(tail -1 "$OUT/pytest_asan.log")"
UPOW_NATIVE_SO=$ROOT/build/native-tsan/_native$EXT TSAN_OPTIONS=halt_on_error=1:report_signal_unsafe=0 \
  timeout -k 10 900 "$OUT/pysan_tsan" -m pytest -q -x -m "not gpu" -p no:cacheprovider \
  tests/test_mempool_index.py tests/test_ledger_writer.py tests/test_log_appender.py tests/test_process_tuning.py \
  > "$OUT/pytest_tsan.log" 2>&1 \
  || { tail -60 "$OUT/pytest_tsan.log"; exit 1; }
echo "python tests under TSan: $(tail -1 "$OUT/pytest_tsan.log")"
echo "sanitize_host: all stages passed"
