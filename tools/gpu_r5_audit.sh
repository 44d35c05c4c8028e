# Per-layer route audit at batch 1024 (tools/conv_roofline.py): 1x1 data gradients and all weight gradients.
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5au}
for m in c1 c3 proj; do
  timeout -k 10 400 python -u tools/conv_roofline.py --batch 1024 --only dgrad --match $m --tiles --tile-list 8,9,12 > gpurun_out/${tag}_dgrad_$m.log 2>&1 || { tail -20 gpurun_out/${tag}_dgrad_$m.log; exit 1; }
  grep -v "amdgpu\|TOTAL" gpurun_out/${tag}_dgrad_$m.log
done
timeout -k 10 500 python -u tools/conv_roofline.py --batch 1024 --only wgrad > gpurun_out/${tag}_wgrad.log 2>&1 || { tail -20 gpurun_out/${tag}_wgrad.log; exit 1; }
grep -v "amdgpu" gpurun_out/${tag}_wgrad.log
