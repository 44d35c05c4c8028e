#!/usr/bin/env python
"""Per-step kernel time summary of a rocprofv3 --stats run: python tools/kstats.py <kernel_stats.csv> <steps> [top]"""
import csv
import sys


def main():
    path, steps = sys.argv[1], float(sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"total kernel time per step: {tot / steps / 1e6:.3f} ms")
    for r in rows[:top]:
        print(f'{float(r["TotalDurationNs"]) / steps / 1e6:8.3f} ms {int(r["Calls"]) / steps:6.1f}x '
              f'{float(r["AverageNs"]) / 1e3:8.1f}us  {r["Name"][:100]}')


if __name__ == "__main__":
    main()
