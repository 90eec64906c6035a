#!/bin/bash
# Build a variant of libfvad.so with extra compile flags (experiments):
#   tools/variant.sh <name> "<EXTRA_HIPFLAGS>"  ->  formula-vad_amd/lib/var/libfvad_<name>.so
# Select it at run time with FVAD_LIB=formula-vad_amd/lib/var/libfvad_<name>.so
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=${1:?name}
W=/tmp/fvad_var_$NAME
rm -rf "$W" && mkdir -p "$W"
cp -r "$ROOT/formula-vad_amd/csrc" "$ROOT/formula-vad_amd/Makefile" "$W/"
mkdir -p "$W/include" && cp "$ROOT/include/fvad.h" "$W/include/"
# the Makefile refers to ../include/fvad.h relative to the package dir
mkdir -p "$W/pkg" && mv "$W/csrc" "$W/Makefile" "$W/pkg/"
make -s -j8 -C "$W/pkg" EXTRA_HIPFLAGS="${2:-}" ${3:-} lib/libfvad.so
mkdir -p "$ROOT/formula-vad_amd/lib/var"
cp "$W/pkg/lib/libfvad.so" "$ROOT/formula-vad_amd/lib/var/libfvad_$NAME.so"
echo "built formula-vad_amd/lib/var/libfvad_$NAME.so"
