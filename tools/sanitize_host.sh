#!/bin/bash
# Build + run the native runtime's host-logic test under AddressSanitizer + UndefinedBehaviorSanitizer
# (CPU only; host code, no GPU code in the binary).  usage: bash tools/sanitize_host.sh [OUT_DIR]
set -e
cd "$(dirname "$0")/.."
OUT=${1:-build/sanitize}
mkdir -p "$OUT"
ROCM=${ROCM_PATH:-/opt/rocm}
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -D__HIP_PLATFORM_AMD__ -I"$ROCM/include" -Icsrc csrc/tests/host_logic_test.cpp -o "$OUT/host_logic_test"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/host_logic_test"
