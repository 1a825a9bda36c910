#!/bin/bash
# Host-side AddressSanitizer + UndefinedBehaviorSanitizer run of the C++ FMI surface: the host test suite
# (threads over Loopback, fork()ed peers over LocalSocket) and the C1 benchmark with 3 forked peers.
# CPU only (no GPU needed). Usage, from the repo root: bash tools/sanitize_host.sh
set -euo pipefail
R=$PWD
OUT=$R/build/asan
mkdir -p "$OUT"
FLAGS="-std=c++17 -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -pthread"
INC="-I$R/fmi_amd/cpp/include -I$R/include"
LIB="-L$R/fmi_amd/lib -lfmi_dev -Wl,-rpath,$R/fmi_amd/lib"
g++ $FLAGS $INC -o "$OUT/test_communicator" "$R/fmi_amd/cpp/tests/test_communicator.cpp" $LIB
g++ $FLAGS $INC -o "$OUT/c1_bench" "$R/fmi_amd/cpp/tools/c1_bench.cpp" $LIB
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 ASAN_OPTIONS=detect_leaks=1
"$OUT/test_communicator"
"$OUT/c1_bench" --reps 3 --mib 4 --peers 3
echo "sanitized host runs: clean"
