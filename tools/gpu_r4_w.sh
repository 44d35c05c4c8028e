# round 4 session W: dS attention path v4 (LDS-DMA ring dQ GEMM): tests, per-kernel times, A/B
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attention.py > gpurun_out/r4w_att.log 2>&1; rc=$?; echo "att rc=$rc"; tail -1 gpurun_out/r4w_att.log; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
DTF_ATTN_DS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4w_p1 -o run -- python3 $R/tools/bench_attention.py > $R/gpurun_out/r4w_p1.log 2>&1; rc=$?; echo "p1 rc=$rc"; [ $rc -lt 124 ] || exit $rc
DTF_ATTN_DS_STAGE=0 DTF_ATTN_DS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4w_p2 -o run -- python3 $R/tools/bench_attention.py > $R/gpurun_out/r4w_p2.log 2>&1; rc=$?; echo "p2 rc=$rc"; [ $rc -lt 124 ] || exit $rc
cd $R
grep -v Warn gpurun_out/r4w_p1.log gpurun_out/r4w_p2.log
for d in p1 p2; do echo "== $d"; python3 - gpurun_out/r4w_$d/run_results.db <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
q = ("select s.display_name, count(*), avg(d.end-d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
     "on d.kernel_id = s.id group by s.display_name")
import collections
q = ("select s.display_name, d.start, d.end from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
     "on d.kernel_id = s.id order by d.start")
per = collections.defaultdict(list)
for n, a, b in c.execute(q):
    if 'attn' in n and 'fwd' not in n:
        per[n.replace('(anonymous namespace)::', '').split('(')[0]].append((b - a) / 1e3)
for n, v in per.items():
    k = len(v) // 4
    print(f"{n:45s}", len(v), [round(sum(v[i*k+2:(i+1)*k]) / (k-2), 1) for i in range(4)])
PY
done
js() { grep '^{"metric"' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$2'", d["value"], d["ms_per_step"], d["config"].get("final_loss"))'; }
for i in 1; do
  timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4w_g1$i.log 2>&1 || exit 1
  DTF_ATTN_DS=0 timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4w_g0$i.log 2>&1 || exit 1
  js gpurun_out/r4w_g1$i.log gpt2_ds; js gpurun_out/r4w_g0$i.log gpt2_nods
done
DTF_ATTN_DS=1 timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/r4w_b1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/r4w_b0.log 2>&1 || exit 1
js gpurun_out/r4w_b1.log bert_ds; js gpurun_out/r4w_b0.log bert_nods
