"""Per-kernel PMC digest of scripts/pmc.sh output (per-wave instruction mix,
wait / activity fractions).  python scripts/pmc_table.py DIR"""
import collections
import csv
import glob
import sys

per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + '/p*/pmc_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        per[r['Kernel_Name'][:70]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, d in per.items():
    s = {c: sum(v) / len(v) for c, v in d.items()}
    w = s.get('SQ_WAVES', 1)
    print(k, 'dispatches', len(d.get('SQ_WAVES', [])))
    print('   waves %.0f VALU/wave %.0f LDS/wave %.0f SALU/wave %.0f VMEM_RD/wave %.1f WR %.1f LDS-conflict/LDS %.2f' % (
        w, s['SQ_INSTS_VALU'] / w, s['SQ_INSTS_LDS'] / w, s['SQ_INSTS_SALU'] / w, s['SQ_INSTS_VMEM_RD'] / w,
        s['SQ_INSTS_VMEM_WR'] / w, s['SQ_LDS_BANK_CONFLICT'] / max(1, s['SQ_INSTS_LDS'])))
    if 'SQ_WAVE_CYCLES' in s:
        wc = s['SQ_WAVE_CYCLES']
        print('   wait_any %.2f wait_inst_any %.2f active_any %.2f active_valu %.3f active_lds %.3f wait_lds %.3f '
              'busy %.0f gui %.0f valu/gui/SIMD %.2f' % (
                  s['SQ_WAIT_ANY'] / wc, s['SQ_WAIT_INST_ANY'] / wc, s['SQ_ACTIVE_INST_ANY'] / wc,
                  s['SQ_ACTIVE_INST_VALU'] / wc, s['SQ_ACTIVE_INST_LDS'] / wc, s['SQ_WAIT_INST_LDS'] / wc,
                  s['SQ_BUSY_CYCLES'], s['GRBM_GUI_ACTIVE'], s['SQ_INSTS_VALU'] / s['GRBM_GUI_ACTIVE'] / 1024))
