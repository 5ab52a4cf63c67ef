#!/bin/bash
# CPU test suite (dry-run handles, design, ABI, oracle) against the host ASan/UBSan build
# (make -C go-audio-resampler_amd asan).  CPU only: GPU sanitizers are not available.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$R/go-audio-resampler_amd" asan
RT=$(/opt/rocm/lib/llvm/bin/clang -print-file-name=libclang_rt.asan-x86_64.so)
export GAR_LIB_PATH="$R/go-audio-resampler_amd/libgar_asan.so"
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$RT" python -m pytest "$R/tests" -q -m "not gpu" -p no:cacheprovider -x ${@:-}
