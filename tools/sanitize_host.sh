#!/usr/bin/env bash
# Build tools/host_selftest.cpp + the native library's host code with ASan + UBSan and run it
# (CPU only: GPU sanitizers are not used). Usage: tools/sanitize_host.sh [outdir]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${1:-build/sanitize}
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
HDRS="csrc/native.h csrc/sha256_common.h csrc/p256_field.h"
if stale "$OUT/p256.o" csrc/p256.hip $HDRS; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Xarch_host -O0 -g1 -std=c++17 -I/opt/rocm/include $SAN_HOST \
    -c csrc/p256.hip -o "$OUT/p256.o"
fi
for f in csrc/sha256_host.cpp csrc/sha256_ni.cpp csrc/base58.cpp csrc/p256_host.cpp tools/host_selftest.cpp; do
  o="$OUT/$(basename "${f%.cpp}").o"
  if stale "$o" "$f" $HDRS; then
    $CXX $CFLAGS -fsanitize=address,undefined -fno-sanitize-recover=undefined -pthread -c "$f" -o "$o"
  fi
done
$CXX -fsanitize=address,undefined -pthread "$OUT"/host_selftest.o "$OUT"/p256.o "$OUT"/sha256_host.o \
  "$OUT"/sha256_ni.o "$OUT"/base58.o "$OUT"/p256_host.o -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -o "$OUT/host_selftest"
# leak checking off: the HIP runtime keeps process-lifetime allocations
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/host_selftest"
# ThreadSanitizer on the host worker pool (csrc/thread_pool.h)
if stale "$OUT/pool_selftest" tools/pool_selftest.cpp csrc/thread_pool.h; then
  $CXX -O1 -g -std=c++17 -fsanitize=thread -pthread -Icsrc tools/pool_selftest.cpp -o "$OUT/pool_selftest"
fi
TSAN_OPTIONS=halt_on_error=1 "$OUT/pool_selftest"
