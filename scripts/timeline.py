"""Print the kernel timeline of the last encode in a rocprofv3 kernel trace
(kernels longer than a threshold), and per-kernel totals per encode."""
import csv, re, sys
path = sys.argv[1]
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.1
r = list(csv.DictReader(open(path)))
r.sort(key=lambda x: int(x['Start_Timestamp']))
def short(n):
    if 'rocprim' in n:
        m = re.findall(r'(onesweep_iteration|onesweep_global_offsets|partition_impl|scan_impl|init_lookback_scan_state_kernel|segmented_sort\w*|segmented\w*|sort_single\w*|warp_sort\w*|block_sort\w*)', n)
        return 'rp:' + (m[0] if m else n[:40])
    return n.split('(')[0][-40:]
idx = [i for i, x in enumerate(r) if 'gather_blocks' in x['Kernel_Name']]
st = idx[-2]
t0 = int(r[st]['Start_Timestamp'])
tot = {}
for x in r[st - 2:]:
    s = int(x['Start_Timestamp']); e = int(x['End_Timestamp'])
    k = short(x['Kernel_Name'])
    tot[k] = tot.get(k, 0) + (e - s) / 1e6
    if (e - s) / 1e6 > thr or 'gather' in k:
        print("%8.3f %8.3f q%s %-45s %s" % ((s - t0) / 1e6, (e - s) / 1e6, x['Queue_Id'], k, x['Grid_Size_X']))
print("end %.3f ms" % ((max(int(x['End_Timestamp']) for x in r[st:]) - t0) / 1e6))
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
    print("%-45s %8.3f" % (k, v))
