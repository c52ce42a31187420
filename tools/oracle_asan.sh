#!/usr/bin/env bash
# Host sanitizers on the CPU oracle (oracle/fmcw_cpu.c): AddressSanitizer + UBSan, run here.
set -euo pipefail
cd "$(dirname "$0")/.."
gcc -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all -fopenmp -std=gnu11 \
    -Wall -Wno-unused-result -o /tmp/oracle_asan tools/oracle_asan.c -lm
ASAN_OPTIONS=detect_leaks=1:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 /tmp/oracle_asan
