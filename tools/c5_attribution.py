"""Attribute every C5 family whose MLProbs output differs from the same
orchestration driving the multi-threaded reference CLIs (verdict r04, item 6;
CPU only, in this container).

For each TEST/ox + TEST/sabre family (tests/golden/sweep.json.xz):
  ours     mlprobs with the aligners in-process on the host context (bit for
           bit the device path: tests/test_pipeline*.py, test_heavy_gpu.py)
  mt       mlprobs driving oracle/_ref/c_p_np_aln (OpenMP on every core) and
           oracle/_ref/quickprobs -t T as external commands -- what
           bench.py's C5 reference leg runs
both at the wall clock (the reference's -p 1 refinement is seeded by
srand(time(0)), CPNP/MSA.cpp, so a -p 1 family matches only when both runs
draw the same second).  Every family whose outputs differ is re-run with the
clock fixed (MLP_SRAND_TIME for ours, oracle/_ref/c_p_np_aln_ft with
REF_FIXED_TIME for the reference):
  ours_ft, st_ft   ours and the reference CLIs single-threaded (c_p_np_aln
                   under taskset -c 0, quickprobs -t 1)
  mt1_ft, mt2_ft   the reference CLIs multi-threaded, twice
and the first stage where the traces part (mlprobs --trace: the -G features
line, classifier 1, the base MSA's column scores, the regions, the realigned
regions, the final MSA) is named for ours vs mt and mt1_ft vs mt2_ft.
Cause per family:
  time-seed      equal with the clock fixed (ours_ft == mt1_ft == mt2_ft)
  race           the two multi-threaded reference runs differ from each other
                 with the clock fixed, and ours_ft equals st_ft (the
                 reference's schedule-dependent BuildPosterior accumulation,
                 CPNP/ProbabilisticModel.h:1223-1283)
  threads        mt1_ft == mt2_ft but != st_ft == ours_ft (deterministic at T
                 threads, a different summation order than one thread)
  UNEXPLAINED    ours_ft != st_ft: a real divergence (to be fixed)

    python tools/c5_attribution.py [--threads 8] [--max-cells 5e7] [--out profiles/r05_c5_attribution.json]
"""
import argparse
import json
import lzma
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..')
BIN = os.path.join(ROOT, 'mlprobs_amd', 'cli', 'mlprobs')
CP = os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln')
CP_FT = os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln_ft')
QP = os.path.join(ROOT, 'oracle', '_ref', 'quickprobs')
FIXED = '1700000000'
STAGES = ('features_line', 'class1', 'col_score', 'regions', 'realigned', 'output')


def wrapper(td, name, body):
    path = os.path.join(td, name)
    with open(path, 'w') as fh:
        fh.write('#!/bin/sh\n' + body + ' "$@"\n')
    os.chmod(path, 0o755)
    return path


def run(fa, td, tag, ref=None, threads=1, fixed=False):
    """ours (ref=None) or the reference CLIs: ref='mt' (c_p_np_aln on every
    core: it sets omp_set_num_threads(omp_get_num_procs()) itself,
    CPNP/MSA.cpp:145-151, so OMP_NUM_THREADS does not bind it; quickprobs -t
    threads) or ref='st' (c_p_np_aln under taskset -c 0, quickprobs -t 1)."""
    out, trace = os.path.join(td, tag + '.msa'), os.path.join(td, tag + '.json')
    env = dict(os.environ, MLP_HOST_MAX_CELLS='1e30', MLP_HOST_THREADS=str(threads))
    cmd = [BIN, '-q', '--trace', trace]
    if ref:
        pre = f'REF_FIXED_TIME={FIXED} exec ' if fixed else 'exec '
        cp = wrapper(td, f'cp_{ref}_{int(fixed)}.sh',
                     pre + ('taskset -c 0 ' if ref == 'st' else '') + (CP_FT if fixed else CP))
        env.update(OMP_WAIT_POLICY='passive')
        cmd += ['--cpnp', cp, '--quickprobs', f'{QP} -t {1 if ref == "st" else threads}', '--tmp', td]
    if fixed:
        env.update(MLP_SRAND_TIME=FIXED)
    r = subprocess.run(cmd + [fa, out], capture_output=True, timeout=3600, env=env)
    if r.returncode != 0 or not os.path.exists(out):
        return None
    with open(out, encoding='latin-1') as fh:
        o = fh.read()
    with open(trace) as fh:
        t = json.load(fh)
    t['output'] = o
    return t


def first_diff(a, b):
    if a is None or b is None:
        return 'failed'
    for k in STAGES:
        if a.get(k) != b.get(k):
            return k
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--threads', type=int, default=8)
    ap.add_argument('--max-cells', type=float, default=5e7)
    ap.add_argument('--out', default=os.path.join(ROOT, 'profiles', 'r05_c5_attribution.json'))
    ap.add_argument('--only', default=None, help='comma-separated family names')
    ap.add_argument('--recheck', default=None,
                    help='a previous output: re-run each differing family\'s multi-threaded reference K more times '
                         'with the clock fixed and reclassify (race = two multi-threaded runs differ)')
    ap.add_argument('--k', type=int, default=4)
    args = ap.parse_args()
    if args.recheck:
        return recheck(args)
    with lzma.open(os.path.join(ROOT, 'tests', 'golden', 'sweep.json.xz'), 'rt') as fh:
        fams = json.load(fh)
    names = [k for k in sorted(fams) if k.split('/')[0] in ('ox', 'sabre')]
    if args.only:
        names = args.only.split(',')
    skipped = [k for k in names if fams[k]['cells'] > args.max_cells]
    names = [k for k in names if fams[k]['cells'] <= args.max_cells]
    rows, same = [], 0
    t0 = time.time()
    with tempfile.TemporaryDirectory() as td:
        for k, name in enumerate(names):
            fa = os.path.join(td, 'f.fa')
            with open(fa, 'wb') as fh:
                fh.write(fams[name]['fa'].encode('latin-1'))
            ours = run(fa, td, 'ours', threads=args.threads)
            mt = run(fa, td, 'mt', ref='mt', threads=args.threads)
            if ours is not None and mt is not None and ours['output'] == mt['output']:
                same += 1
            else:
                ours_ft = run(fa, td, 'ours_ft', threads=args.threads, fixed=True)
                st_ft = run(fa, td, 'st_ft', ref='st', threads=1, fixed=True)
                mt1 = run(fa, td, 'mt1_ft', ref='mt', threads=args.threads, fixed=True)
                mt2 = run(fa, td, 'mt2_ft', ref='mt', threads=args.threads, fixed=True)
                o_ft = ours_ft and ours_ft['output']
                if o_ft is None or st_ft is None or o_ft != st_ft['output']:
                    cause = 'UNEXPLAINED'
                elif mt1 and mt2 and o_ft == mt1['output'] == mt2['output']:
                    cause = 'time-seed'
                elif mt1 and mt2 and mt1['output'] != mt2['output']:
                    cause = 'race'
                else:
                    cause = 'threads'
                rows.append({'family': name, 'cells': fams[name]['cells'], 'class1': ours and ours.get('class1'),
                             'path': ours and ours.get('path'), 'first_stage_ours_vs_mt': first_diff(ours, mt),
                             'first_stage_mt1_vs_mt2_fixed_clock': first_diff(mt1, mt2),
                             'first_stage_ours_vs_st_fixed_clock': first_diff(ours_ft, st_ft),
                             'first_stage_st_vs_mt1_fixed_clock': first_diff(st_ft, mt1), 'cause': cause})
                print(json.dumps(rows[-1]), flush=True)
            if k % 25 == 0:
                print(f'# {k + 1}/{len(names)} families, {len(rows)} differ, {time.time() - t0:.0f} s',
                      file=sys.stderr, flush=True)
    causes = {}
    for r in rows:
        causes[r['cause']] = causes.get(r['cause'], 0) + 1
    res = {'families': len(names), 'identical': same, 'differing': len(rows), 'causes': causes,
           'skipped_above_max_cells': skipped, 'threads': args.threads,
           'method': __doc__.split('\n\n')[1].replace('\n', ' '), 'rows': rows}
    with open(args.out, 'w') as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ('rows', 'method')}))


def recheck(args):
    """Second pass over the differing families: the reference CLIs
    multi-threaded K times and single-threaded once, clock fixed, against ours
    (clock fixed).  Causes: race (the multi-threaded runs disagree among
    themselves at some stage), threads (they agree with each other, not with
    the single-threaded run), time-seed (all agree with ours and the family
    takes the -p 1 path: the wall-clock difference is srand(time(0))),
    race-unreproduced (all agree, -p 0 path: the wall-clock multi-threaded run
    differed, the K fixed-clock ones did not), UNEXPLAINED (ours differs from
    the single-threaded reference)."""
    with open(args.recheck) as fh:
        prev = json.load(fh)
    with lzma.open(os.path.join(ROOT, 'tests', 'golden', 'sweep.json.xz'), 'rt') as fh:
        fams = json.load(fh)
    rows = []
    with tempfile.TemporaryDirectory() as td:
        for r in prev['rows']:
            name = r['family']
            fa = os.path.join(td, 'f.fa')
            with open(fa, 'wb') as fh:
                fh.write(fams[name]['fa'].encode('latin-1'))
            ours = run(fa, td, 'ours_ft', threads=args.threads, fixed=True)
            st = run(fa, td, 'st_ft', ref='st', threads=1, fixed=True)
            mts = [run(fa, td, f'mt{k}_ft', ref='mt', threads=args.threads, fixed=True) for k in range(args.k)]
            ok = ours is not None and st is not None and all(m is not None for m in mts)
            stages_mt = sorted({first_diff(mts[0], m) for m in mts[1:]} - {None}, key=STAGES.index) if ok else []
            if not ok or ours['output'] != st['output']:
                cause = 'UNEXPLAINED'
            elif stages_mt:
                cause = 'race'
            elif mts[0]['output'] != st['output']:
                cause = 'threads'
            elif (ours.get('class1') == 1):
                cause = 'time-seed'
            else:
                cause = 'race-unreproduced'
            distinct = len({m['output'] for m in mts}) if ok else None
            row = dict(r, cause=cause, mt_runs=args.k, mt_distinct_outputs=distinct,
                       mt_distinct_features=len({m['features_line'] for m in mts}) if ok else None,
                       mt_stages_that_vary=stages_mt,
                       first_stage_ours_vs_st_fixed_clock=first_diff(ours, st),
                       first_stage_st_vs_mt_fixed_clock=sorted({first_diff(st, m) for m in mts} - {None},
                                                               key=STAGES.index) if ok else None)
            rows.append(row)
            print(json.dumps(row), flush=True)
    causes = {}
    for r in rows:
        causes[r['cause']] = causes.get(r['cause'], 0) + 1
    res = dict(prev, causes=causes, rows=rows, recheck={'k': args.k, 'method': recheck.__doc__.replace('\n', ' ')})
    with open(args.out, 'w') as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ('rows', 'method', 'recheck')}))


if __name__ == '__main__':
    main()
