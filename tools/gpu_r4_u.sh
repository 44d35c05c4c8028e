# round 4 session U: dS attention path v2 (tiled dS, coalesced rowsum, 2-deep dQ prefetch): tests, per-kernel times, A/B
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_attention.py > gpurun_out/r4u_att.log 2>&1; rc=$?; echo "att rc=$rc"; tail -1 gpurun_out/r4u_att.log; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
DTF_ATTN_DS=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r4u_p1 -o run -- python3 $R/tools/bench_attention.py > $R/gpurun_out/r4u_p1.log 2>&1; rc=$?; echo "p1 rc=$rc"; [ $rc -lt 124 ] || exit $rc
cd $R
grep -v Warn gpurun_out/r4u_p1.log
python3 - gpurun_out/r4u_p1/run_results.db <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
q = ("select s.display_name, count(*), avg(d.end-d.start) from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
     "on d.kernel_id = s.id group by s.display_name")
for n, cnt, avg in sorted(c.execute(q), key=lambda r: -r[1] * r[2]):
    if 'attn' in n: print(f"{cnt:5d} {avg/1e3:8.1f}us {n[:100]}")
PY
js() { grep '^{"metric"' $1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$2'", d["value"], d["ms_per_step"], d["config"].get("final_loss"))'; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4u_g1$i.log 2>&1 || exit 1
  DTF_ATTN_DS=0 timeout -k 10 300 python bench.py --model gpt2_medium --steps 10 --warmup 3 > gpurun_out/r4u_g0$i.log 2>&1 || exit 1
  js gpurun_out/r4u_g1$i.log gpt2_ds; js gpurun_out/r4u_g0$i.log gpt2_nods
done
DTF_ATTN_DS=1 timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/r4u_b1.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --model bert_base --steps 10 --warmup 3 > gpurun_out/r4u_b0.log 2>&1 || exit 1
js gpurun_out/r4u_b1.log bert_ds; js gpurun_out/r4u_b0.log bert_nods
