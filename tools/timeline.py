#!/usr/bin/env python
"""Step timeline of a rocprofv3 --kernel-trace run: python tools/timeline.py <kernel_trace.csv> [steps] [top]

Splits the trace into steps at the optimizer kernel (the last kernel of a train step), then reports per step:
wall time, the union of kernel-busy intervals (any stream), per-stream busy time, GPU-idle gaps (no kernel
running on any stream) bucketed by the kernel that ends right before the gap, and the kernels that run while
the main stream is idle. Used to tell launch/host gaps from kernel time before optimising kernels."""
import collections
import csv
import sys


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r.get("Stream_Id") or r.get("Queue_Id") or "0"))
    rows.sort()
    return rows


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    path = sys.argv[1]
    want = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
    rows = load(path)
    ends = [i for i, r in enumerate(rows) if "optim_kernel" in r[2]]
    if len(ends) < 2:
        print("fewer than 2 optimizer kernels in the trace")
        return
    steps = list(zip(ends[:-1], ends[1:]))[-want:]
    gap_by = collections.Counter()
    gap_n = collections.Counter()
    for a, b in steps:
        seg = rows[a + 1:b + 1]
        t0, t1 = rows[a][1], rows[b][1]
        busy = union([(s, e) for s, e, _, _ in seg])
        per = collections.defaultdict(list)
        for s, e, n, q in seg:
            per[q].append((s, e))
        print(f"step wall {(t1 - t0) / 1e6:.3f} ms  kernels {len(seg)}  gpu-busy(any stream) {busy / 1e6:.3f} ms  "
              f"idle {(t1 - t0 - busy) / 1e6:.3f} ms  " +
              "  ".join(f"stream {q}: {union(v) / 1e6:.3f} ms ({len(v)})" for q, v in sorted(per.items())))
        # idle gaps: time with no kernel on any stream
        last_end, last_name = t0, rows[a][2]
        for s, e, n, q in seg:
            if s > last_end:
                gap_by[last_name[:90]] += s - last_end
                gap_n[last_name[:90]] += 1
            if e > last_end:
                last_end, last_name = e, n
    k = len(steps)
    print(f"\nGPU-idle gaps per step by the kernel that precedes them (top {top}):")
    for name, t in gap_by.most_common(top):
        print(f"  {t / k / 1e3:9.1f} us  {gap_n[name] / k:6.1f}x  {name}")


if __name__ == "__main__":
    main()
