#!/usr/bin/env python
"""Steady-state kernel statistics of a rocprofv3 --kernel-trace run.

    python tools/steady_stats.py <kernel_trace.csv> [--skip 1] [--top 30] [--marker optim_kernel]

The trace is cut into training steps at the last kernel of each step (the fused optimizer, `--marker`); the first
`--skip` steps after the first marker (warm-up effects, one-time set-up copies, fp8 scale bootstrap) and everything
before the first marker are dropped, so every figure is per STEADY step (total/7 mixed the first
step's set-up work into the per-step numbers). Reports:
  * per-kernel ms/step, calls/step and mean duration over the kept steps;
  * the per-stream split (stream 0 = the main / data-gradient chain = the critical path);
  * for every main-stream kernel, the share of its run time during which another stream also had a kernel running
    (how much of it overlapped the weight-gradient side stream);
  * copy/fill kernels per step (attribution of __amd_rocclr_* work).
"""
import argparse
import bisect
import collections
import csv


def load(path):
    rows = []
    if path.endswith(".db"):  # rocprofv3's default rocpd (SQLite) output
        import sqlite3
        c = sqlite3.connect(path)
        q = ("select d.start, d.end, s.display_name, d.stream_id, d.queue_id from rocpd_kernel_dispatch d "
             "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        for st, en, name, sid, qid in c.execute(q):
            rows.append((int(st), int(en), name, str(sid if sid is not None else qid)))
        rows.sort()
        return rows
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r.get("Stream_Id") or r.get("Queue_Id") or "0"))
    rows.sort()
    return rows


def merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(s, e, merged, starts):
    """Length of [s, e) covered by the merged interval list."""
    i = max(0, bisect.bisect_right(starts, s) - 1)
    tot = 0
    while i < len(merged) and merged[i][0] < e:
        a, b = merged[i]
        tot += max(0, min(b, e) - max(a, s))
        i += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=1)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--marker", default="optim_kernel")
    ap.add_argument("--width", type=int, default=100)
    a = ap.parse_args()
    rows = load(a.trace)
    ends = [i for i, r in enumerate(rows) if a.marker in r[2]]
    # a step ends at its LAST marker kernel (a per-bucket update issues several): keep markers that are followed by
    # a non-marker kernel on the main stream before the next marker
    step_ends = [i for k, i in enumerate(ends) if k + 1 == len(ends) or ends[k + 1] != i + 1]
    if len(step_ends) < a.skip + 2:
        raise SystemExit(f"only {len(step_ends)} steps in the trace")
    first, last = step_ends[a.skip], step_ends[-1]
    seg = rows[first + 1:last + 1]
    nsteps = len(step_ends) - 1 - a.skip
    wall = rows[last][1] - rows[first][1]
    streams = sorted({r[3] for r in seg}, key=lambda q: (len(q), q))
    main_q = collections.Counter(r[3] for r in seg if "gemm" in r[2] or "bn_" in r[2]).most_common(1)[0][0]
    per_name = collections.defaultdict(lambda: [0, 0])
    per_stream = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0]))
    for s, e, n, q in seg:
        per_name[n][0] += e - s
        per_name[n][1] += 1
        per_stream[q][n][0] += e - s
        per_stream[q][n][1] += 1
    busy = merge([(s, e) for s, e, _, _ in seg])
    print(f"# steady state: {nsteps} steps after skipping {a.skip}; wall {wall / nsteps / 1e6:.3f} ms/step; "
          f"GPU busy (any stream) {sum(b - s for s, b in busy) / nsteps / 1e6:.3f} ms/step")
    tot = sum(v[0] for v in per_name.values())
    print(f"total kernel time per step: {tot / nsteps / 1e6:.3f} ms")
    for n, (t, c) in sorted(per_name.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"{t / nsteps / 1e6:8.3f} ms {c / nsteps:6.1f}x {t / c / 1e3:8.1f}us  {n[:a.width]}")
    others = {q: merge([(s, e) for s, e, _, qq in seg if qq != q]) for q in streams}
    print("\n# per stream (main = the stream carrying most GEMM/BN kernels; 'ovl' = share of the kernel's time during "
          "which another stream was also running a kernel)")
    for q in streams:
        items = per_stream[q]
        qt = sum(v[0] for v in items.values())
        print(f"stream {q}{' (main)' if q == main_q else ''} total {qt / nsteps / 1e6:.2f} ms/step")
        om = others[q]
        starts = [x[0] for x in om]
        ov = collections.Counter()
        for s, e, n, qq in seg:
            if qq == q:
                ov[n] += overlap(s, e, om, starts)
        for n, (t, c) in sorted(items.items(), key=lambda kv: -kv[1][0])[:a.top]:
            print(f"   {t / nsteps / 1e6:7.3f} ms {c / nsteps:6.1f}x  ovl {100.0 * ov[n] / max(1, t):5.1f}%  "
                  f"{n[:a.width - 10]}")
    copies = {n: v for n, v in per_name.items() if n.startswith("__amd_rocclr")}
    if copies:
        print("\n# runtime copy / fill kernels per steady step")
        for n, (t, c) in sorted(copies.items(), key=lambda kv: -kv[1][1]):
            print(f"   {c / nsteps:6.1f}x {t / nsteps / 1e3:8.1f} us  {n}")


if __name__ == "__main__":
    main()
