# round 4 session C2b: fp8 GEMM roles on hipBLASLt (bit mask) and the bf16 forward projections on hipBLASLt: A/B
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
js() { grep '^{"metric"' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$2'", d["value"], d["ms_per_step"], d["config"].get("final_loss"))'; }
for i in 1 2; do
  for m in 0 4 3 7; do
    DTF_FP8_BLASLT=$m timeout -k 10 300 python bench.py --model gpt2_medium_fp8 --steps 10 --warmup 3 > gpurun_out/r4c2_f$m$i.log 2>&1 || { tail -20 gpurun_out/r4c2_f$m$i.log; exit 1; }
    js gpurun_out/r4c2_f$m$i.log fp8_mask$m
  done
done
for i in 1 2; do
  for b in 0 1; do
    DTF_BLAS_FWD=$b timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4c2_g$b$i.log 2>&1 || exit 1
    js gpurun_out/r4c2_g$b$i.log gpt2_blasfwd$b
    DTF_BLAS_FWD=$b timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/r4c2_b$b$i.log 2>&1 || exit 1
    js gpurun_out/r4c2_b$b$i.log bert_blasfwd$b
  done
done
