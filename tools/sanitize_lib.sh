#!/bin/bash
# The library's host logic under AddressSanitizer, on the CPU: the C-ABI tests that need no GPU
# (schedules for up to 2,000 peers, argument validation, LOCAL / PROC communicator bookkeeping, tuning)
# against build/asan_lib/libfmi_dev.so (make -C fmi_amd/csrc asan: -fsanitize=address on the host
# compilation only). Python is not instrumented, so the sanitizer runtime is preloaded and leak checking
# (Python's own allocations) is off. Usage, from the repo root: bash tools/sanitize_lib.sh
set -euo pipefail
R=$PWD
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
test -f "$R/build/asan_lib/libfmi_dev.so" || make -C "$R/fmi_amd/csrc" asan
FMI_DEV_LIB=$R/build/asan_lib/libfmi_dev.so LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 \
  python -m pytest "$R/tests/test_abi.py" -q -p no:cacheprovider
echo "sanitized library host logic: clean"
