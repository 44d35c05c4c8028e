#!/bin/bash
# Build the host runtime + csrc/runtime/selftest.cc under sanitizers and run it (host code only:
# GPU sanitizers are not available on the MI355X pool).
#   asan: AddressSanitizer + UndefinedBehaviorSanitizer (g++)
#   tsan: ThreadSanitizer (clang from /opt/rocm/lib/llvm: gcc 11's libtsan misses pthread_cond_clockwait,
#         which libstdc++ uses for condition_variable::wait_for, and reports false double-locks)
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$R/build/sanitize}
mkdir -p "$OUT"
SRC="$R/csrc/runtime/crc32c.cc $R/csrc/runtime/tensor_bundle.cc $R/csrc/runtime/event_writer.cc $R/csrc/runtime/kv_store.cc $R/csrc/runtime/ps_transport.cc $R/csrc/runtime/shm_allreduce.cc $R/csrc/runtime/selftest.cc"
CLANG=/opt/rocm/lib/llvm/bin/clang++
g++ -std=c++17 -O1 -g -fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer \
    -msse4.2 -I"$R/csrc/runtime" $SRC -o "$OUT/selftest_asan" -lpthread -lrt
ASAN_OPTIONS=detect_leaks=1 "$OUT/selftest_asan" "$OUT"
if [ -x "$CLANG" ]; then
  "$CLANG" -std=c++17 -O1 -g -fsanitize=thread -msse4.2 -I"$R/csrc/runtime" $SRC -o "$OUT/selftest_tsan" -lpthread -lrt
  TSAN_OPTIONS=halt_on_error=1 "$OUT/selftest_tsan" "$OUT"
fi
echo "sanitizers clean"
