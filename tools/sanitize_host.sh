#!/bin/bash
# Host-code sanitizer run (CPU only, no device): the file parsers the `cnn`
# CLI feeds with user data -- JPEG / PNG / PNM decoders and the JSON reader --
# built with AddressSanitizer + UndefinedBehaviorSanitizer and driven by the
# deterministic mutation fuzzer host/test/codec_fuzz.cpp over seed files.
#   tools/sanitize_host.sh [--iters N] SEED...   (default seeds: tests/golden)
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
H=$R/cnn-super-resolution_amd/host
O=${SANITIZE_OUT:-$R/cnn-super-resolution_amd/build/sanitize}
mkdir -p "$O"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
  -I"$R/include" -I"$H/src" "$H/test/codec_fuzz.cpp" "$H/src/Image.cpp" "$H/src/Jpeg.cpp" "$H/src/Json.cpp" "$H/src/Config.cpp" \
  -o "$O/codec_fuzz" -lz
args=()
seeds=()
while [ $# -gt 0 ]; do
  case "$1" in
    --iters|--seed) args+=("$1" "$2"); shift 2;;
    *) seeds+=("$1"); shift;;
  esac
done
if [ ${#seeds[@]} -eq 0 ]; then
  seeds=("$R/tests/golden/color_grid2.jpg" "$R/tests/golden/config/"*.json)
fi
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$O/codec_fuzz" "${args[@]}" "${seeds[@]}"
