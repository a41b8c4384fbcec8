"""bench.py's printed line stays small enough for the driver to parse.

Round 5's line grew to ~20 KB (every end-to-end run's stage split, the C5
slowest list, repeated sub-dicts) and the driver recorded `parsed: null`.
The line is now a compact summary (bench.compact_line) with the full record
in a side file; these tests hold it under 10 KB for the host dry run, for a
full single-GPU record (round 5's own, profiles/r05_final4_bench.json) and
for an eight-rank record.
"""
import copy
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIMIT = 10000


def _bench():
    spec = importlib.util.spec_from_file_location('bench_mod', os.path.join(ROOT, 'bench.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_host_dry_run_line_parses(tmp_path):
    detail = str(tmp_path / 'detail.json')
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--host', '--nseq', '10', '--len', '40', '--steps', '1',
           '--warmup', '0', '--no-cpu', '--no-e2e', '--no-qp', '--no-shards', '--relax', '1']
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd='/tmp',
                       env=dict(os.environ, MLP_BENCH_DETAIL=detail))
    assert r.returncode == 0, r.stderr[-3000:]
    last = r.stdout.strip().splitlines()[-1]
    assert len(last) < LIMIT
    d = json.loads(last)
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'config', 'roofline',
              'cpu_baseline', 'relax'):
        assert k in d
    assert d['detail'] == detail
    with open(detail) as fh:
        full = json.load(fh)
    assert full['value'] == d['value'] and full['relax']['rounds'] == 1


def test_full_single_gpu_record_compacts():
    b = _bench()
    with open(os.path.join(ROOT, 'profiles', 'r05_final4_bench.json')) as fh:
        out = json.load(fh)
    # round 5's record plus what this round's legs add: the per-family
    # differences of the C5 leg
    out['c5_pipeline']['differing'] = [{'name': f'ox/fam{k:03d}', 'path': 'RIR', 'first_stage': 'features_line',
                                        'cause': 'race' if k % 3 else 'unexplained: reference reproducible'} for k in range(40)]
    line = b.compact_line(out)
    s = json.dumps(line)
    assert len(s) < b.LINE_LIMIT < LIMIT
    for k in ('roofline', 'cpu_baseline', 'parity', 'relax', 'quickprobs', 'e2e', 'c5_pipeline',
              'virtual_shards', 'kernels_ms_per_step', 'stage_roofline'):
        assert k in line, k
    assert line['value'] == out['value'] and line['ms_per_step'] == out['ms_per_step']
    assert line['roofline']['valu_issue']['frac'] > 0
    assert line['c5_pipeline']['differing']['n'] == 40
    assert line['e2e']['C3 512x400']['posterior_stage']['pair_cells_per_s'] > 0


def test_eight_rank_record_compacts():
    b = _bench()
    rank = {'rank': 0, 'pairs': 16352, 'pair_cells': 2628239257, 'step_ms': 70.1, 'gather_ms': 20.2,
            'posterior_ms': 49.9, 'gather_bytes_in': 3124643817, 'gather_GBps': 154.7,
            'kernels_ms_per_step': {'forward': 23.1, 'backward': 30.3, 'local_totals': 8.1,
                                    'merge_mea_sparsify': 10.9, 'compact': 0.5, 'allgather': 20.2},
            'roofline': {'bound': 'hbm', 'kernel': 'backward', 'achieved': 2100.1, 'peak': 8000.0, 'unit': 'GB/s',
                         'frac': 0.2625, 'avg_launch_ms': 30.3, 'algo_bytes_per_cell': 24},
            'store_hash': 'f' * 64}
    out = {'metric': 'm', 'value': 3.1e11, 'unit': 'pair-cells/s', 'n_gpus': 8, 'steps': 20, 'warmup': 5,
           'ms_per_step': 70.1, 'config': {'workload': 'C3'}, 'roofline': rank['roofline'], 'cpu_baseline': None,
           'parity': None, 'ranks': [dict(copy.deepcopy(rank), rank=r) for r in range(8)],
           'relax': {'rounds': 1, 'seconds': 0.2,
                     'per_round': [{'seconds': 0.2, 'gather_ms': 5.0, 'nnz_out': 173924262,
                                    'ranks': [{'rank': r, 'seconds': 0.2, 'relax_kernel_ms': 150.0, 'gather_ms': 5.0,
                                               'store_hash': 'e' * 64} for r in range(8)]}]}}
    line = b.compact_line(out)
    assert len(json.dumps(line)) < b.LINE_LIMIT
    assert len(line['ranks']) == 8 and len(line['relax']['per_round'][0]['ranks']) == 8
