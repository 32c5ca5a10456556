#!/bin/bash
# Build a tuning variant of libldgpu.so: tools/build_variant.sh TAG "-DMACRO=..."
# -> spark-languagedetector_amd/lib/libldgpu_TAG.so (select with LDGPU_LIB=...).
set -eu
cd "$(dirname "$0")/../spark-languagedetector_amd"
TAG=$1; shift
make -s -j8 BUILD=build_$TAG LIBOUT=lib/libldgpu_$TAG.so EXTRA="$*" lib/libldgpu_$TAG.so
