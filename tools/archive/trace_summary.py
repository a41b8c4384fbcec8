"""Per-dispatch durations (ms) of the sweep kernels from a rocprofv3 kernel
trace: one line per kernel name, dispatches in launch order."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
by = defaultdict(list)
for r in rows:
    n = r['Kernel_Name'].split('(')[0].replace('void mlp::', '')
    by[n].append(((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6,
                  int(r['Grid_Size_X']) // 64, int(r['VGPR_Count']), int(r['LDS_Block_Size'])))
for n, v in by.items():
    print('%-40s n=%d total %.1f ms waves %s vgpr %d lds %d' % (n, len(v), sum(x[0] for x in v),
          ' '.join('%.1f/%d' % (x[0], x[1]) for x in v[-6:]), v[0][2], v[0][3]))
