#!/bin/bash
# Host-code AddressSanitizer + UBSan run of vtk_host.cpp (CPU only; no GPU code is sanitized).
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p tools/bin
/opt/rocm/bin/hipcc --offload-arch=gfx950 -std=c++17 -O1 -g -ffp-contract=off -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
    -fno-omit-frame-pointer tools/asan_host.cpp vt-precondition_amd/csrc/vtk_host.cpp -o tools/bin/asan_host -lpthread
ASAN_OPTIONS=detect_leaks=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 tools/bin/asan_host
