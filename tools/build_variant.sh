#!/bin/bash
# Build a variant of libia.so with extra compile definitions for A/B runs on the GPU box
# (tools/gpu.sh ablib / IA_LIB_PATH): _ab/libia_NAME.so from a copy of the sources.
#   tools/build_variant.sh NAME -DMACRO=V [...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
rm -rf _ab/csrc && mkdir -p _ab && cp -r image-analogies-python_amd/csrc _ab/csrc && rm -rf _ab/csrc/_build
make -s -C _ab/csrc -j8 OUT=../libia_$name.so HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result $*" > /dev/null
grep -A12 "Function Name: _ZN2ia11k_screen16pILi11ELb0E" _ab/csrc/_build/ia_screen16.res | grep -E "VGPRs:|Scratch" | sed "s/^/$name: /"
