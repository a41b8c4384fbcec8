"""Per-kernel sums of one tools/valu_ab.sh pass: VALU, SALU and LDS
instructions (wave-level) per C3 pair-cell of the kernel's launches."""
import csv
import glob
import re
import sys
from collections import defaultdict

CELLS = 21025914059   # C3 pair-cells of one step (bench.py config.pair_cells)


def main(d, tag):
    f = glob.glob(f'{d}/**/p_counter_collection.csv', recursive=True)
    tot = defaultdict(lambda: defaultdict(float))
    with open(f[0]) as fh:
        for r in csv.DictReader(fh):
            m = re.search(r'mlp::(k_[a-z_]+)(<[^>]*>)?', r['Kernel_Name'])
            k = (m.group(1) + (m.group(2) or '')) if m else r['Kernel_Name'][:30]
            tot[k][r['Counter_Name']] += float(r['Counter_Value'])
    for k in sorted(tot, key=lambda k: -tot[k].get('SQ_INSTS_VALU', 0)):
        c = tot[k]
        if c.get('SQ_INSTS_VALU', 0) < 1e9:
            continue
        print(f"{tag:8s} {k:28s} VALU/cell {c['SQ_INSTS_VALU'] / CELLS:6.3f} SALU/cell {c.get('SQ_INSTS_SALU', 0) / CELLS:6.3f} "
              f"LDS/cell {c.get('SQ_INSTS_LDS', 0) / CELLS:6.3f}")


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
