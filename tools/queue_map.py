"""Which HIP hardware queue every stream's kernels went to, from a rocprofv3 --kernel-trace database (rocpd SQLite):
a stream that shares another stream's in-order queue serialises with it (HIP maps streams onto at most
GPU_MAX_HW_QUEUES queues per process, 4 by default).

    python tools/queue_map.py <run_results.db> [--steps N]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    q = ("select d.stream_id, d.queue_id, count(*), sum(d.end - d.start) from rocpd_kernel_dispatch d "
         "group by d.stream_id, d.queue_id order by d.stream_id, d.queue_id")
    by_stream = collections.defaultdict(list)
    for sid, qid, n, ns in c.execute(q):
        by_stream[sid].append((qid, n, ns / 1e6))
    print("stream -> queue (kernels, kernel ms over the whole run)")
    for sid, rows in sorted(by_stream.items()):
        print(f"  stream {sid}: " + ", ".join(f"queue {qid} ({n} kernels, {ms:.1f} ms)" for qid, n, ms in rows))
    queues = collections.defaultdict(set)
    for sid, rows in by_stream.items():
        for qid, _, _ in rows:
            queues[qid].add(sid)
    shared = {q: s for q, s in queues.items() if len(s) > 1}
    print("queues shared by several streams:", shared if shared else "none")


if __name__ == "__main__":
    main()
