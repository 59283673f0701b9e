#!/bin/bash
# Build a variant of libia.so with extra compile definitions for A/B runs on the GPU box
# (tools/gpu.sh ablib / IA_LIB_PATH): _ab/libia_NAME.so from a copy of the sources.
#   tools/build_variant.sh NAME -DMACRO=V [...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
rm -rf _ab/csrc && mkdir -p _ab && cp -r image-analogies-python_amd/csrc _ab/csrc && rm -rf _ab/csrc/_build
# EXTRA (not HIPFLAGS): a command-line HIPFLAGS would override the Makefile's per-object
# screen flags (-fno-honor-nans, -amdgpu-mfma-vgpr-form=1) and handicap every variant
make -s -C _ab/csrc -j8 OUT=../libia_$name.so EXTRA="$*" > /dev/null
grep -A12 "Function Name: _ZN2ia12_GLOBAL__N_111k_screen16rILi11E" _ab/csrc/_build/ia_screen16r.res | grep -E "VGPRs:|Scratch" | sed "s/^/$name: /"
