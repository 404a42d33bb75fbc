#!/bin/bash
# Build kernel tuning variants of libaeon_hip.so into aeon_amd/variants/ (select one with
# AEON_HIP_LIB=aeon_amd/variants/<name>.so).  Usage: tools/build_variants.sh name="-DX=1 ..." ...
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$R/aeon_amd/variants"
for spec in "$@"; do
  name="${spec%%=*}"; defs="${spec#*=}"
  make -s -C "$R/aeon_amd/csrc" OUT="$R/aeon_amd/variants/$name.so" BUILD="$R/aeon_amd/csrc/build_$name" KDEFS="$defs" -j4 "$R/aeon_amd/variants/$name.so"
done
