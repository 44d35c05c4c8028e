#!/usr/bin/env python
"""Every kernel of ONE steady training step of a rocprofv3 --kernel-trace run, in issue order per stream: start offset,
duration, stream, grid, name — to attribute per-layer time (which conv call of which stage is slow), which the
per-kernel-name aggregates of tools/steady_stats.py cannot.

    python tools/step_list.py <kernel_trace.csv> [--marker optim_kernel] [--step 2]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="optim_kernel")
    ap.add_argument("--step", type=int, default=2, help="which step (counted in markers) to list")
    args = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(args.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     r.get("Stream_Id") or r.get("Queue_Id") or "0", r.get("Grid_Size", "")))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if args.marker in r[2]]
    if len(marks) < args.step + 1:
        raise SystemExit(f"only {len(marks)} marker kernels")
    lo, hi = marks[args.step - 1] + 1, marks[args.step] + 1
    t0 = rows[lo][0]
    print(f"# step {args.step}: {hi - lo} kernels, wall {(rows[hi - 1][1] - t0) / 1e6:.3f} ms")
    for s, e, name, sid, grid in rows[lo:hi]:
        print(f"{(s - t0) / 1e3:10.1f} us {(e - s) / 1e3:9.1f} us  s{sid:>3s}  g{grid:>9s}  {name[:110]}")


if __name__ == "__main__":
    main()
