"""Per-stream timeline of a rocprofv3 kernel trace (rocpd .db): busy time,
idle gaps and the kernels around the largest gaps, and how much of the wall
time 0 / 1 / 2+ streams had a kernel running.

python scripts/ktimeline.py RUN_results.db [--skip 0.3] [--gaps 12]
(--skip: fraction of the trace's wall time dropped at the start: warmup)"""
import argparse
import sqlite3
from collections import defaultdict


def short(n):
    n = n.split("(")[0]
    return n.replace("void ", "").replace("lfm::", "")[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--skip", type=float, default=0.3)
    ap.add_argument("--gaps", type=int, default=12)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select stream_id, name, start, end from kernels order by start").fetchall()
    t0 = min(r[2] for r in rows)
    t1 = max(r[3] for r in rows)
    cut = t0 + a.skip * (t1 - t0)
    rows = [r for r in rows if r[2] >= cut]
    wall = (t1 - cut) / 1e6
    per = defaultdict(list)
    for sid, name, s, e in rows:
        per[sid].append((s, e, name))
    print("window %.1f ms, %d kernels, %d streams" % (wall, len(rows), len(per)))
    for sid, ks in sorted(per.items()):
        busy = sum(e - s for s, e, _ in ks) / 1e6
        gaps = []
        for (s0, e0, n0), (s1, e1, n1) in zip(ks, ks[1:]):
            if s1 > e0:
                gaps.append(((s1 - e0) / 1e6, n0, n1))
        tg = sum(g for g, _, _ in gaps)
        print("stream %s: %d kernels busy %.1f ms (%.0f%%) gaps %.1f ms (%d)" %
              (sid, len(ks), busy, 100 * busy / wall, tg, len(gaps)))
        agg = defaultdict(lambda: [0, 0.0])
        for g, n0, n1 in gaps:
            k = (short(n0), short(n1))
            agg[k][0] += 1
            agg[k][1] += g
        for (n0, n1), (cnt, tot) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.gaps]:
            print("   %7.2f ms in %4d gaps  %s -> %s" % (tot, cnt, n0, n1))
    # concurrency: events sweep
    ev = []
    for sid, ks in per.items():
        for s, e, _ in ks:
            ev.append((s, 1, sid))
            ev.append((e, -1, sid))
    ev.sort()
    act = defaultdict(int)
    lvl = defaultdict(float)
    last = cut
    for t, d, sid in ev:
        n = sum(1 for v in act.values() if v > 0)
        lvl[min(n, 3)] += (t - last) / 1e6
        last = t
        act[sid] += d
    print("streams active: " + ", ".join("%d: %.1f ms" % (k, v) for k, v in sorted(lvl.items())))


if __name__ == "__main__":
    main()
