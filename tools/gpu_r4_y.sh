# round 4 session Y: XCD-aware block order in every attention kernel: tests, per-kernel times (both backward paths),
# GPT-2 / BERT end to end
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attention.py > gpurun_out/r4y_att.log 2>&1; rc=$?; echo "att rc=$rc"; tail -1 gpurun_out/r4y_att.log; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
n=0
for e in "DTF_ATTN_DS=1" "DTF_ATTN_DS=0"; do
  n=$((n+1))
  env $e timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4y_p$n -o run -- python3 $R/tools/bench_attention.py > $R/gpurun_out/r4y_p$n.log 2>&1; rc=$?; echo "p$n [$e] rc=$rc"; [ $rc -lt 124 ] || exit $rc
  grep "bwd" $R/gpurun_out/r4y_p$n.log
  python3 - $R/gpurun_out/r4y_p$n/run_results.db <<'PY'
import collections, sqlite3, sys
c = sqlite3.connect(sys.argv[1])
q = ("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
     "on d.kernel_id = s.id order by d.start")
per = collections.defaultdict(list)
for n, a, b in c.execute(q):
    if 'attn' in n:
        per[n.replace('(anonymous namespace)::', '').split('(')[0]].append((b - a) / 1e3)
for n, v in per.items():
    k = len(v) // 4 if len(v) >= 48 else len(v) // 2
    parts = 4 if len(v) >= 48 else 2
    print(f"  {n:45s}", len(v), [round(sum(v[i*k+2:(i+1)*k]) / (k-2), 1) for i in range(parts)])
PY
done
cd $R
js() { grep '^{"metric"' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$2'", d["value"], d["ms_per_step"], d["config"].get("final_loss"))'; }
for m in gpt2_medium bert_base gpt2_medium_fp8; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 > gpurun_out/r4y_$m.log 2>&1 || exit 1
  js gpurun_out/r4y_$m.log $m
done
DTF_ATTN_DS=0 timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4y_g0.log 2>&1 || exit 1
js gpurun_out/r4y_g0.log gpt2_nods
