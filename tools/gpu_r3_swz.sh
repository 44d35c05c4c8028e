#!/bin/bash
# GPU session: gemm256 tests, PMC of the BERT FFN1 GEMMs, BERT-base / GPT-2-medium benches.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu -k "gemm or fp8 or dense or linear or bert or gpt" > $OUT/t_swz.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" $OUT/t_swz.log | head -20; tail -5 $OUT/t_swz.log; exit 1; }
tail -1 $OUT/t_swz.log
bash tools/gpu_r3_pmcgemm.sh > /dev/null 2>&1 || { echo "pmc failed"; exit 1; }
grep -E "gemm256|bank-conflict|WAIT_INST_LDS /|MFMA busy" $OUT/pmcg_summary.txt
MODELS="bert_base gpt2_medium gpt2_medium_fp8" bash tools/gpu_r3_xfmr.sh | grep -v "dropout="
