# Per-layer conv forward at batch 1024: default route vs forced 128-row LDS-DMA tiles / conv256 (tools/conv_roofline.py).
# bash tools/gpu_r5_croof.sh <tag> <match> [tiles]
set -o pipefail
mkdir -p gpurun_out
tag=${1:-r5cr}; match=${2:-c2}; tiles=${3:-8,9,11,12,14}
timeout -k 10 500 python -u tools/conv_roofline.py --batch 1024 --only fwd --match $match --tiles --tile-list $tiles > gpurun_out/${tag}_fwd.log 2>&1 || { tail -20 gpurun_out/${tag}_fwd.log; exit 1; }
cat gpurun_out/${tag}_fwd.log
