set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in main p0a3 p1a2 p0a2 main2; do
  if [ $v = main ] || [ $v = main2 ]; then unset IA_LIB_PATH; else export IA_LIB_PATH=$PWD/_ab/libia_$v.so; fi
  echo "== $v" >> gpurun_out/abpc.txt
  timeout -k 10 200 python -u tools/screen_img_bench.py --M 342,256,128 --reps 20 --forms s0,pc >> gpurun_out/abpc.txt 2>&1 || exit 1
done
cat gpurun_out/abpc.txt | grep -v amdgpu.ids
