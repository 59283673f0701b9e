#!/bin/bash
# A/B of k_screen16p build variants (tools/build_variant.sh) on the c4 finest-level screen:
# time per form and the per-stage stamps (tools/screen_img_bench.py --trace).
#   tools/ab_screen.sh VARIANT [VARIANT ...]      (run through gpurun)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
    echo "== $v" >> gpurun_out/ab_screen.txt
    IA_LIB_PATH=$PWD/_ab/libia_$v.so timeout -k 10 200 python -u tools/screen_img_bench.py --M 342,128 \
        --reps 20 --forms pc --trace >> gpurun_out/ab_screen.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/ab_screen.txt
