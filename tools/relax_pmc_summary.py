"""Per-launch PMC summary of tools/relax_pmc.sh output: python tools/relax_pmc_summary.py DIR"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
for f in sorted(glob.glob(f'{d}/p*/p_counter_collection.csv')):
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = (r['Kernel_Name'][:40], r['Counter_Name'])
        agg[k] += float(r['Counter_Value'])
        disp[k].add(r['Dispatch_Id'])
    for k in sorted(agg):
        print(f'{k[0]:42s} {k[1]:22s} {agg[k] / len(disp[k]):.4e}')
for f in sorted(glob.glob(f'{d}/p1/p_kernel_trace.csv')):
    for r in csv.DictReader(open(f)):
        if 'relax' in r['Kernel_Name']:
            print(r['Kernel_Name'][:40], 'LDS', r['LDS_Block_Size'], 'VGPR', r['VGPR_Count'], 'SGPR', r['SGPR_Count'],
                  'wg', r.get('Workgroup_Size_X', r.get('Workgroup_Size', '?')),
                  'ms', (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
