#!/bin/bash
# Host-side sanitizer runs (CPU only; GPU ASan is not available on this pool):
# the C-ABI library's loader / WAV / tokenizer code (tests/test_capi.py,
# malformed files included) under clang's ASan + UBSan, and the oracle
# (tests/test_oracle.py) under gcc's.  Leak checks are off (the Python
# interpreter itself is not instrumented).
set -e -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
make -s -C "$R/whisper.rs_amd/csrc" asan
make -s -C "$R/oracle" asan
CLANG_RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
cd "$R"
LD_PRELOAD="$CLANG_RT" WMI_LIB="$R/whisper.rs_amd/_asan/libwhisper_mi355x.so" \
  python3 -m pytest -q -p no:cacheprovider tests/test_capi.py tests/test_audio_text.py -m "not gpu"
LD_PRELOAD="$(gcc -print-file-name=libasan.so):$(gcc -print-file-name=libubsan.so)" \
  WMI_ORACLE_LIB="$R/oracle/_asan/liboracle.so" \
  python3 -m pytest -q -p no:cacheprovider tests/test_oracle.py tests/test_quant.py -m "not gpu"
