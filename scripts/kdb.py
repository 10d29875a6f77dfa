"""Per-kernel summary of a rocprofv3 kernel-trace database (rocpd .db).

python scripts/kdb.py RUN_results.db [--top 40] [--match name] [--csv out.csv]
"""
import argparse
import sqlite3
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--match", default="")
    ap.add_argument("--csv", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels").fetchall()
    agg = defaultdict(list)
    for name, s, e in rows:
        if a.match and a.match not in name:
            continue
        agg[name.split("(")[0][:90]].append((e - s) / 1e6)
    tot = sum(sum(v) for v in agg.values())
    out = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    lines = ["name,calls,total_ms,avg_ms,min_ms,max_ms,pct"]
    for k, v in out[:a.top]:
        lines.append("%s,%d,%.3f,%.4f,%.4f,%.4f,%.1f" % (k.replace(",", ";"), len(v), sum(v), sum(v) / len(v), min(v),
                                                     max(v), 100 * sum(v) / tot))
    print("\n".join(lines))
    if a.csv:
        open(a.csv, "w").write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
