# round 4 session B2b: hipBLASLt fp8 (torch._scaled_mm) per role at the GPT-2-medium projection shapes
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/probe_scaled_mm.py > gpurun_out/r4b2_smm.log 2>&1; echo "rc=$?"
grep -v Warn gpurun_out/r4b2_smm.log
