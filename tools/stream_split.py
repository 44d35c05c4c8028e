#!/usr/bin/env python
"""Per-stream kernel time of a rocprofv3 --kernel-trace run: python tools/stream_split.py <kernel_trace.csv> <steps>

Which kernels sit on the main (data-gradient) stream and which on the weight-gradient side stream, per step.
Kernels of the two streams overlap on the GPU, so their per-stream sums exceed the wall time; the main stream's
busy time is the critical path."""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = float(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
    d = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        k = (r["Stream_Id"], r["Kernel_Name"][:90])
        d[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[k][1] += 1
    for s in sorted({k[0] for k in d}):
        items = sorted([(v[0], k[1], v[1]) for k, v in d.items() if k[0] == s], reverse=True)
        print("stream", s, "total %.2f ms/step" % (sum(i[0] for i in items) / steps / 1e6))
        for t, n, c in items[:top]:
            print("   %7.3f ms %6.1fx %s" % (t / steps / 1e6, c / steps, n))


if __name__ == "__main__":
    main()
