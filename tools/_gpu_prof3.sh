set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for m in bert_base gpt2_medium_fp8; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/prof_$m -o run -- python3 $R/bench.py --model $m --steps 3 --warmup 2 > $R/gpurun_out/prof_$m.log 2>&1 || { echo PROFFAIL; tail -5 $R/gpurun_out/prof_$m.log; exit 1; }
done
echo ok
