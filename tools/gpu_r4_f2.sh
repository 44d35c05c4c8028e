# round 4 session F2b: host issue time per step with the fp8 forward / data-gradient GEMMs on hipBLASLt
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for m in 7 4 7 4; do
  DTF_FP8_BLASLT=$m timeout -k 10 300 python bench.py --model gpt2_medium_fp8 --steps 10 --warmup 3 > gpurun_out/r4f2_b$m.log 2>&1 || exit 1
  grep '^{"metric"' gpurun_out/r4f2_b$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("mask '$m'", d["value"], d["ms_per_step"], "host_issue_ms", d.get("host_issue_ms_per_step"), d.get("host_issue_ms_single_step"))'
done
for m in gpt2_medium_fp8 gpt2_medium bert_base; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 --graph 1 > gpurun_out/r4f2_g$m.log 2>&1 || { echo "$m graph failed"; tail -5 gpurun_out/r4f2_g$m.log; continue; }
  grep '^{"metric"' gpurun_out/r4f2_g$m.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("graph '$m'", d["value"], d["ms_per_step"], d["config"].get("hipgraph"), d["config"].get("final_loss"), "host", d.get("host_issue_ms_single_step"))'
done
