"""Kernel time against gaps in a rocprofv3 trace database (rocpd, the default output of
``rocprofv3 --kernel-trace``): the dispatches of one kernel in time order, cut into runs wherever
the GPU was idle for more than --split-ms; per run the launches, queues, mean kernel duration,
mean gap between a launch's end and the next one's start, and the fraction of the run's span the
kernel was executing (overlapping launches on several queues counted once).

  python tools/trace_gaps.py <results.db> [--kernel mgj_search] [--split-ms 1] [--candidates N]"""
import argparse
import glob
import json
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--kernel", default="mgj_search")
    ap.add_argument("--split-ms", type=float, default=1.0)
    ap.add_argument("--candidates", type=int, default=0, help="candidates per launch (for a rate)")
    a = ap.parse_args()
    path = a.db if a.db.endswith(".db") else glob.glob(a.db + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(path)
    rows = c.execute("select start, end, queue_id from kernels where name like ? order by start",
                     (f"%{a.kernel}%",)).fetchall()
    runs, cur = [], []
    last_end = None
    for s, e, q in rows:
        if last_end is not None and s - last_end > a.split_ms * 1e6:
            runs.append(cur)
            cur = []
        cur.append((s, e, q))
        last_end = e if last_end is None else max(last_end, e)
    if cur:
        runs.append(cur)
    for r in runs:
        span = max(e for _, e, _ in r) - r[0][0]
        busy, edge = 0, r[0][0]  # union of [start, end) intervals
        for s, e, _ in r:
            if e > edge:
                busy += e - max(s, edge)
                edge = e
        gaps = [max(0, r[k + 1][0] - r[k][1]) for k in range(len(r) - 1)]
        rec = {"kernel": a.kernel, "launches": len(r), "queues": len({q for _, _, q in r}),
               "mean_kernel_us": round(sum(e - s for s, e, _ in r) / len(r) / 1e3, 2),
               "mean_gap_us": round(sum(gaps) / len(gaps) / 1e3, 2) if gaps else None,
               "span_ms": round(span / 1e6, 4), "kernel_busy_frac": round(busy / span, 4) if span else None}
        if a.candidates:
            rec["candidates_per_s_span"] = a.candidates * len(r) / (span * 1e-9)
            rec["candidates_per_s_kernel"] = a.candidates / (sum(e - s for s, e, _ in r) / len(r) * 1e-9)
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
