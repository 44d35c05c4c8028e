set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu > gpurun_out/t_all.log 2>&1 || { echo TESTFAIL; tail -40 gpurun_out/t_all.log; exit 1; }
tail -n 1 gpurun_out/t_all.log
for m in bert_base gpt2_medium_fp8; do
timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/b1_$m.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/b1_$m.log; exit 1; }
tail -n 1 gpurun_out/b1_$m.log | cut -c1-160
DTF_GLDS_DENSE=0 timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/b0_$m.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/b0_$m.log; exit 1; }
tail -n 1 gpurun_out/b0_$m.log | cut -c1-160
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log | cut -c1-160
