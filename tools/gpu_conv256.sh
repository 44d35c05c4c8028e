#!/bin/bash
# GPU session: conv kernel tests, then the ResNet-50 conv roofline: default (old) kernels + forced conv256 variants.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv" > $OUT/convtests.log 2>&1 || { echo "conv tests failed"; grep -E "FAIL|Error|assert|error" $OUT/convtests.log | head -30; tail -5 $OUT/convtests.log; exit 1; }
tail -1 $OUT/convtests.log
DTF_CONV256=0 timeout -k 10 600 python tools/conv_roofline.py --tiles --tile-list ${TL:-11,12,13,14} > $OUT/roof_tiles.txt 2>&1 || { echo "roofline failed"; tail -5 $OUT/roof_tiles.txt; exit 1; }
tail -4 $OUT/roof_tiles.txt
