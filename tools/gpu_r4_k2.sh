# round 4 session K2: host-side (Python) profile of the GPT-2-medium fp8 and bf16 steps
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for m in gpt2_medium_fp8 gpt2_medium; do
  timeout -k 10 300 python -m cProfile -o gpurun_out/r4k2_$m.prof bench.py --model $m --steps 8 --warmup 3 > gpurun_out/r4k2_$m.log 2>&1 || exit 1
  python - gpurun_out/r4k2_$m.prof <<'PY'
import pstats, sys
p = pstats.Stats(sys.argv[1])
p.sort_stats("tottime").print_stats(28)
PY
done
