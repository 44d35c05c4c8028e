# round 4 session H2: fp8 GEMM roles on hipBLASLt again after the host-time fixes (2 interleaved rounds)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for i in 1 2; do
  for m in 4 3 7 0; do
    DTF_FP8_BLASLT=$m timeout -k 10 300 python bench.py --model gpt2_medium_fp8 --steps 10 --warmup 3 > gpurun_out/r4h2_f$m$i.log 2>&1 || exit 1
    grep '^{"metric"' gpurun_out/r4h2_f$m$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("mask '$m'", d["value"], d["ms_per_step"], "host", d.get("host_issue_ms_single_step"), d["config"].get("final_loss"))'
  done
done
timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4h2_g.log 2>&1 || exit 1
grep '^{"metric"' gpurun_out/r4h2_g.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bf16", d["value"], d["ms_per_step"], "host", d.get("host_issue_ms_single_step"))'
