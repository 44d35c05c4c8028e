#!/usr/bin/env python
"""Kernel-by-kernel difference of two steady_stats.py reports (B - A, ms/step):

    python tools/kdiff.py stats_a.txt stats_b.txt [--min 0.02]
"""
import argparse
import re


def load(path):
    d, head = {}, ""
    for line in open(path):
        if not head:
            head = line.strip()
        m = re.match(r"\s+([\d.]+) ms\s+([\d.]+)x\s+([\d.]+)us\s+(.*)", line)
        if m and m.group(4)[:90] not in d:  # the first (whole-step) table only
            d[m.group(4)[:90]] = (float(m.group(1)), float(m.group(2)))
        if line.startswith("# per stream"):
            break
    return head, d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("a")
    ap.add_argument("b")
    ap.add_argument("--min", type=float, default=0.02)
    o = ap.parse_args()
    ha, a = load(o.a)
    hb, b = load(o.b)
    print("A:", ha)
    print("B:", hb)
    z = (0.0, 0.0)
    rows = sorted(((b.get(k, z)[0] - a.get(k, z)[0], k) for k in set(a) | set(b)))
    for dlt, k in rows:
        if abs(dlt) >= o.min:
            print(f"{dlt:+.3f} ms  A {a.get(k, z)[0]:.3f} ({a.get(k, z)[1]:.0f}x)  B {b.get(k, z)[0]:.3f} "
                  f"({b.get(k, z)[1]:.0f}x)  {k}")
    print(f"total kernel time B - A: {sum(v[0] for v in b.values()) - sum(v[0] for v in a.values()):+.3f} ms")


if __name__ == "__main__":
    main()
