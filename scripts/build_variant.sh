#!/bin/bash
# Build libvtkrylov.so with extra compile flags into tools/bin/lib_<name>/ (A/B runs on the
# GPU box via VTK_LIB; scripts/gpu_steps.sh "variants").
#   scripts/build_variant.sh b "-mcumode"   (the library has no compile-time switches since round 5)
set -eu
cd "$(dirname "$0")/../vt-precondition_amd/csrc"
name=$1; flags=${2:-}
make -s -j8 OBJDIR=../../tools/bin/obj_$name OUT=../../tools/bin/lib_$name/libvtkrylov.so EXTRA="$flags"
echo "built tools/bin/lib_$name ($flags)"
