set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu > gpurun_out/t_all.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_all.log; exit 1; }
tail -n 2 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo BENCHFAIL; tail -20 gpurun_out/bench.log; exit 1; }
tail -n 1 gpurun_out/bench.log
timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/bench_bert.log 2>&1 || { echo BERTFAIL; tail -20 gpurun_out/bench_bert.log; exit 1; }
tail -n 1 gpurun_out/bench_bert.log
timeout -k 10 300 python bench.py --model gpt2_medium_fp8 --steps 10 --warmup 3 > gpurun_out/bench_gpt2.log 2>&1 || { echo GPTFAIL; tail -20 gpurun_out/bench_gpt2.log; exit 1; }
tail -n 1 gpurun_out/bench_gpt2.log
timeout -k 10 300 python tools/conv_roofline.py > gpurun_out/rf_all.log 2>&1
tail -n 4 gpurun_out/rf_all.log
