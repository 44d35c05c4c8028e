# round 4 session Z: full GPU suite, smoke, ResNet-50 bench (eager x2, hipGraph), steady-state kernel stats,
# transformer benches
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
step() {
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $R/gpurun_out/r4z_$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"
  if [ $rc -ge 124 ]; then echo "stopping after $n"; exit $rc; fi
}
step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread
grep -E "passed|failed" gpurun_out/r4z_tests.log | tail -2
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tail -1 gpurun_out/r4z_smoke.log
step b1 300 python bench.py
step b2 300 python bench.py
step bg 300 python bench.py --graph 1
cd /tmp && export TMPDIR=/tmp
step prof 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4z_prof -o run -- python3 $R/bench.py --steps 10 --warmup 5
cd $R
python tools/steady_stats.py gpurun_out/r4z_prof/run_results.db --top 45 > gpurun_out/r4z_steady.txt 2>&1 || true
head -4 gpurun_out/r4z_steady.txt
for m in bert_base gpt2_medium gpt2_medium_fp8; do step $m 300 python bench.py --model $m --steps 10 --warmup 3; done
for f in b1 b2 bg bert_base gpt2_medium gpt2_medium_fp8; do grep '^{"metric"' gpurun_out/r4z_$f.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$f'", d["value"], d["ms_per_step"], d["config"].get("final_loss"), d.get("host_issue_ms_single_step"))'; done
