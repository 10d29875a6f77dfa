"""Kernel timeline of one encode in a rocprofv3 kernel trace.

python scripts/timeline.py TRACE.csv [ENCODE_INDEX=-1] [THRESHOLD_MS=0.1]
An encode starts at a pair of rle1_crc launches (one per HIP stream / batch)
and ends at the last compact_streams before the next encode.  Prints every
kernel longer than the threshold (start, duration, queue) and the per-kernel
totals of that encode."""
import csv
import re
import sys

path = sys.argv[1]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
thr = float(sys.argv[3]) if len(sys.argv) > 3 else 0.1
r = list(csv.DictReader(open(path)))
r.sort(key=lambda x: int(x['Start_Timestamp']))


def short(n):
    if 'rocprim' in n:
        m = re.findall(r'(onesweep_iteration|onesweep_global_offsets|partition_impl|scan_impl|'
                       r'init_lookback_scan_state_kernel|segmented_sort\w*|segmented\w*|sort_single\w*|'
                       r'warp_sort\w*|block_sort\w*)', n)
        return 'rp:' + (m[0] if m else n[:40])
    return n.split('(')[0][-40:]


starts = [i for i, x in enumerate(r) if 'rle1_crc' in x['Kernel_Name']]
groups = [starts[i] for i in range(0, len(starts), 2)]
st = groups[which]
en = groups[which + 1] if which != -1 and which + 1 < len(groups) else len(r)
t0 = int(r[st]['Start_Timestamp'])
tot = {}
last = t0
for x in r[st:en]:
    s = int(x['Start_Timestamp'])
    e = int(x['End_Timestamp'])
    k = short(x['Kernel_Name'])
    if 'bzd' in k or 'unpredict' in k:
        continue
    last = max(last, e)
    tot[k] = tot.get(k, 0) + (e - s) / 1e6
    if (e - s) / 1e6 > thr:
        print("%8.3f %8.3f q%s %-45s %s" % ((s - t0) / 1e6, (e - s) / 1e6, x['Queue_Id'], k, x['Grid_Size_X']))
print("end %.3f ms" % ((last - t0) / 1e6))
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
    print("%-45s %8.3f" % (k, v))
