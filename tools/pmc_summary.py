"""Summarise rocprofv3 PMC passes (tools/pmc_run.sh) per kernel.

FETCH_SIZE is reported in KB and, on gfx950, counts half the bytes of wide
coalesced streaming reads (MI355X_MICROARCH.md, HBM section): we report both
the raw value and the x2-corrected one; WRITE_SIZE is taken as is.

    python tools/pmc_summary.py DIR [per-kernel.json] [traffic.json]

traffic.json (read by bench.py) holds, per bench kernel group (the HIP-event
timed launch groups of bench.py), the measured HBM bytes and VALU wave
instructions per pair-cell of the profiled run, so bench.py can scale them
to its own launches.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r'mlp::(k_[a-z_]+)(<[^>]*>)?', name)
    return (m.group(1) + (m.group(2) or '')) if m else name[:30]


def load(path):
    rows = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            k = short(r['Kernel_Name'])
            rows[k][r['Counter_Name']] += float(r['Counter_Value'])
            calls[k].add(r['Dispatch_Id'])
    return rows, {k: len(v) for k, v in calls.items()}


def main(d):
    res = defaultdict(dict)
    for p in ('p1', 'p2', 'p3'):
        f = os.path.join(d, p, f'{p}_counter_collection.csv')
        if not os.path.exists(f):
            continue
        rows, calls = load(f)
        for k, cs in rows.items():
            res[k].update(cs)
            res[k]['calls'] = calls[k]
    stats = os.path.join(d, 'stats', 'stats_kernel_stats.csv')
    if os.path.exists(stats):
        with open(stats) as fh:
            for r in csv.DictReader(fh):
                k = short(r['Name'])
                res[k]['avg_ns'] = float(r['AverageNs'])
                res[k]['total_ns'] = float(r['TotalDurationNs'])
    out = {}
    for k, c in res.items():
        if 'total_ns' not in c:
            continue
        n = max(c.get('calls', 1), 1)
        e = dict(c)
        if 'FETCH_SIZE' in c:
            e['fetch_bytes_per_launch_raw'] = c['FETCH_SIZE'] * 1024 / n
            e['fetch_bytes_per_launch_x2'] = 2 * c['FETCH_SIZE'] * 1024 / n
        if 'WRITE_SIZE' in c:
            e['write_bytes_per_launch'] = c['WRITE_SIZE'] * 1024 / n
        if 'SQ_WAVE_CYCLES' in c and c['SQ_WAVE_CYCLES']:
            e['valu_active_frac'] = c.get('SQ_ACTIVE_INST_VALU', 0) / c['SQ_WAVE_CYCLES']
            e['wait_any_frac'] = c.get('SQ_WAIT_ANY', 0) / c['SQ_WAVE_CYCLES']
            e['wait_inst_frac'] = c.get('SQ_WAIT_INST_ANY', 0) / c['SQ_WAVE_CYCLES']
        out[k] = e
    return out


GROUPS = {'forward': ('k_forward',), 'backward': ('k_backward', 'k_fold_totals'),
          'local_totals': ('k_local_totals', 'k_local_bounds', 'k_local_list', 'k_local_fold', 'k_local_btot'),
          'merge_mea_sparsify': ('k_merge',), 'compact': ('k_compact',)}


def groups(o, d):
    """Per bench kernel group: bytes and VALU instructions per pair-cell."""
    cells = None
    nnz_in = None  # relaxation round 1 input entries (bench --relax 1)
    for log in ('p1.log', 'p2.log', 'p3.log', 'stats.log'):
        f = os.path.join(d, log)
        if not os.path.exists(f):
            continue
        for line in open(f):
            if line.startswith('{"metric"'):
                b = json.loads(line)
                cells = b['config']['pair_cells'] * (b['steps'] + b['warmup'])
                if b.get('relax') and b['relax']['rounds'] == 1:
                    r0 = b['relax']['per_round'][0]
                    nnz_in = r0['nnz_in'] if 'nnz_in' in r0 else b['relax']['nnz_per_round'][0]
        if cells:
            break
    out = {'_source': os.path.basename(os.path.normpath(d)), '_pair_cells': cells,
           '_note': 'read bytes = 2 x FETCH_SIZE (gfx950 correction), write bytes = WRITE_SIZE'}
    for g, pre in GROUPS.items():
        ks = [k for k in o if k.startswith(pre)]
        if not ks or not cells:
            continue
        rd = sum(o[k].get('fetch_bytes_per_launch_x2', 0) * o[k].get('calls', 1) for k in ks)
        wr = sum(o[k].get('write_bytes_per_launch', 0) * o[k].get('calls', 1) for k in ks)
        vi = sum(o[k].get('SQ_INSTS_VALU', 0) for k in ks)
        ns = sum(o[k]['total_ns'] for k in ks)
        out[g] = {'kernels': ks, 'read_bytes_per_cell': rd / cells, 'write_bytes_per_cell': wr / cells,
                  'traffic_bytes_per_cell': (rd + wr) / cells, 'valu_insts_per_cell': vi / cells,
                  'profiled_ms': ns / 1e6}
    # the consistency round's tile and row-task kernels, per input entry
    ks = [k for k in o if k.startswith('k_relax') and not k.startswith('k_relax_blockmfma')]
    if ks and nnz_in:
        rd = sum(o[k].get('fetch_bytes_per_launch_x2', 0) * o[k].get('calls', 1) for k in ks)
        wr = sum(o[k].get('write_bytes_per_launch', 0) * o[k].get('calls', 1) for k in ks)
        out['relax'] = {'kernels': ks, 'nnz_in': nnz_in, 'read_bytes_per_nnz_in': rd / nnz_in,
                        'write_bytes_per_nnz_in': wr / nnz_in, 'traffic_bytes_per_nnz_in': (rd + wr) / nnz_in,
                        'valu_insts_per_nnz_in': sum(o[k].get('SQ_INSTS_VALU', 0) for k in ks) / nnz_in,
                        'profiled_ms': sum(o[k]['total_ns'] for k in ks) / 1e6}
    return out


if __name__ == '__main__':
    o = main(sys.argv[1])
    for k, e in sorted(o.items(), key=lambda kv: -kv[1]['total_ns']):
        print(f"{k:28s} {e['total_ns']/1e6:8.1f} ms  VALU {e.get('valu_active_frac', 0):.2f} "
              f"waitany {e.get('wait_any_frac', 0):.2f} waitinst {e.get('wait_inst_frac', 0):.2f} "
              f"valuinst {e.get('SQ_INSTS_VALU', 0):.3g} salu {e.get('SQ_INSTS_SALU', 0):.3g} lds {e.get('SQ_INSTS_LDS', 0):.3g} "
              f"rd/launch {e.get('fetch_bytes_per_launch_x2', 0)/1e9:.2f} GB wr/launch {e.get('write_bytes_per_launch', 0)/1e9:.2f} GB")
    if len(sys.argv) > 2:
        with open(sys.argv[2], 'w') as fh:
            json.dump(o, fh, indent=1)
    if len(sys.argv) > 3:
        with open(sys.argv[3], 'w') as fh:
            json.dump(groups(o, sys.argv[1]), fh, indent=1)
