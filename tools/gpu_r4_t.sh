# round 4 session T: per-kernel attention backward times (rocprofv3 kernel stats) for both backward paths
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
DTF_ATTN_DS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4t_p1 -o run -- python3 $R/tools/bench_attention.py > $R/gpurun_out/r4t_p1.log 2>&1; rc=$?; echo "p1 rc=$rc"; [ $rc -lt 124 ] || exit $rc
DTF_ATTN_DS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4t_p0 -o run -- python3 $R/tools/bench_attention.py > $R/gpurun_out/r4t_p0.log 2>&1; rc=$?; echo "p0 rc=$rc"; [ $rc -lt 124 ] || exit $rc
cd $R
for d in p1 p0; do f=$(find gpurun_out/r4t_$d -name "*kernel_stats.csv" | head -1); echo "== $d"; python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if 'attn' in r['Name']:
        print(f"{int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:110]}")
PY
done
js() { grep '^{"metric"' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$2'", d["value"], d["ms_per_step"], d["config"].get("final_loss"))'; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4t_g1$i.log 2>&1 || exit 1
  DTF_ATTN_DS=0 timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4t_g0$i.log 2>&1 || exit 1
  js gpurun_out/r4t_g1$i.log gpt2_ds; js gpurun_out/r4t_g0$i.log gpt2_nods
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_resnet_gpu.py tests/test_model_training_gpu.py > gpurun_out/r4t_tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r4t_tests.log
