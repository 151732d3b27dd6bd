#!/usr/bin/env bash
# Build and run the native host runtime (csrc/native: parser, hashing, java random,
# quantile summaries) under AddressSanitizer + UndefinedBehaviorSanitizer and under
# ThreadSanitizer (the parser is multi-threaded). Host code only: GPU sanitizers are not
# used on this platform. Exit status != 0 on any sanitizer report or failed check.
set -euo pipefail
cd "$(dirname "$0")/.."
out=${OUT:-build/sanitize}
mkdir -p "${out}"
srcs="csrc/native/hash.cpp csrc/native/parser.cpp csrc/native/jrandom.cpp csrc/native/wquantile.cpp csrc/native/tests/native_stress.cpp"
common="-std=c++17 -O1 -g -fno-omit-frame-pointer -pthread -include algorithm"
g++ ${common} -fsanitize=address,undefined -fno-sanitize-recover=all ${srcs} -o "${out}/stress_asan"
g++ ${common} -fsanitize=thread ${srcs} -o "${out}/stress_tsan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 "${out}/stress_asan"
TSAN_OPTIONS=halt_on_error=1 setarch "$(uname -m)" -R "${out}/stress_tsan"
echo "sanitizers clean"
