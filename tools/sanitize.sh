#!/bin/bash
# Host-code sanitizer run (CPU only, no GPU involved):
#   1. the oracle (oracle/src/oracle.cpp) with AddressSanitizer + UndefinedBehaviorSanitizer;
#   2. the product library with ASan + UBSan on its HOST code only (-Xarch_host: the .cli
#      loader, the scene / BVH builder, the host photon-map build, the C ABI; device code is
#      compiled as usual and never runs here);
#   3. the CPU test suite (pytest -m "not gpu") against both, with the clang ASan runtime
#      preloaded into the Python process (both libraries are clang-built so they share it).
# Leak checking is off: CPython and numpy keep allocations alive at exit by design.
#   tools/sanitize.sh [pytest args...]        (outputs under build/san/)
set -eo pipefail
REPO=$(cd "$(dirname "$0")/.." && pwd)
OUT=$REPO/build/san
mkdir -p "$OUT"
CLANG=/opt/rocm/lib/llvm/bin/clang++
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g"

# 1. oracle: the Makefile's flags, clang instead of gcc (one ASan runtime in the process)
$CLANG -O1 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fopenmp $SAN -shared \
  -o "$OUT/liboracle_san.so" "$REPO/oracle/src/oracle.cpp" -L/opt/rocm/lib/llvm/lib -Wl,-rpath,/opt/rocm/lib/llvm/lib

# 2. product library, host-side sanitizers (each -fsanitize= right after -Xarch_host)
python3 - "$OUT/libdistraytracer_san.so" <<'EOF'
import sys
sys.path.insert(0, ".")
from distraytracer_old_amd import build
flags = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
         "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer"]
build.build(defines=flags, out=sys.argv[1])
EOF

# 3. the CPU suite over the sanitized libraries
cd "$REPO"
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
ORACLE_LIB="$OUT/liboracle_san.so" DISTRAYTRACER_LIB="$OUT/libdistraytracer_san.so" \
LD_PRELOAD="$RT" python3 -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@" 2>&1 | tee "$OUT/sanitize.log"
