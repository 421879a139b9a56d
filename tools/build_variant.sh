#!/bin/bash
# build a libsod.so variant with extra -D flags into tools/variants/lib<name>.so
#   tools/build_variant.sh <name> "-DFOO=1 -DBAR=2"
set -e
cd "$(dirname "$0")/../sift-based-od_amd/csrc"
make -s -j8 OBJDIR=../../tools/variants/build_$1 OUT=../../tools/variants/lib$1.so EXTRA="$2"
