"""GPU busy fraction of the last encode in a rocprofv3 kernel trace: union of
kernel intervals (any queue) from the last encode's first predictor launch to
its last kernel, plus the longest idle gaps.  python scripts/busy.py TRACE.csv"""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
r.sort(key=lambda x: int(x['Start_Timestamp']))
starts = [i for i, x in enumerate(r) if 'predict_ring' in x['Kernel_Name']]
i0 = starts[-1]
iv = [(int(x['Start_Timestamp']), int(x['End_Timestamp']), x['Kernel_Name'].split('(')[0][-40:]) for x in r[i0:]]
t0, t1 = iv[0][0], max(e for _, e, _ in iv)
busy, cur_s, cur_e, gaps = 0, None, None, []
for s, e, k in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_e - t0, k))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print("window %.3f ms, busy %.3f ms (%.1f %%), %d gaps" % ((t1 - t0) / 1e6, busy / 1e6, 100 * busy / (t1 - t0), len(gaps)))
for g, at, k in sorted(gaps, reverse=True)[:12]:
    print("  gap %.3f ms at %.3f ms before %s" % (g / 1e6, at / 1e6, k))
