# round 4 session A2: GPT-2-medium bf16 and fp8 steady-state kernel stats
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for m in gpt2_medium_fp8 gpt2_medium; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4a2_$m -o run -- python3 $R/bench.py --model $m --steps 8 --warmup 3 > $R/gpurun_out/r4a2_$m.log 2>&1; rc=$?; echo "$m rc=$rc"; [ $rc -lt 124 ] || exit $rc
  python3 $R/tools/steady_stats.py $R/gpurun_out/r4a2_$m/run_results.db --top 40 --marker optim_kernel > $R/gpurun_out/r4a2_${m}_steady.txt 2>&1 || true
  head -30 $R/gpurun_out/r4a2_${m}_steady.txt | cut -c1-130
done
