#!/bin/bash
# Host code under AddressSanitizer + UBSan, CPU only:
#   * the oracle (clang -fsanitize=address,undefined) and the host translation units of
#     libmq_aead.so (hipcc -Xarch_host -fsanitize=...; kernels unchanged) are rebuilt as `make asan`;
#   * the whole CPU test suite (pytest -m "not gpu") runs against those builds (MQ_ASAN=1) with
#     clang's ASan runtime preloaded into the Python process;
#   * tests/csrc/test_runtime.cpp (device bookkeeping) runs under g++'s sanitizers inside the suite.
# Log: profiles/<tag>_asan_cpu_tests.log. Never run on the GPU box (GPU ASan is not available there).
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
TAG="${1:-r03}"
make -C "$ROOT/oracle" -s asan
make -C "$ROOT/milli_quic_amd/csrc" -s asan
RT="$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -n1)"
LOG="$ROOT/profiles/${TAG}_asan_cpu_tests.log"
{
  echo "# $(date -u +%FT%TZ) host ASan+UBSan CPU suite; runtime $RT"
  echo "# oracle: $ROOT/oracle/build/asan/*.so; libmq_aead: $ROOT/milli_quic_amd/asan/libmq_aead.so"
} > "$LOG"
cd "$ROOT"
# detect_leaks=0: CPython itself does not free everything at exit; ASan still reports every
# out-of-bounds access, use-after-free and UB in the instrumented libraries (halt on the first)
env MQ_ASAN=1 LD_PRELOAD="$RT" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
    UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    python -m pytest tests/ -q -m "not gpu" -p no:cacheprovider 2>&1 | tee -a "$LOG"
