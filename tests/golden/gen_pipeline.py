"""Golden fixtures for the MLProbs pipeline driver (mlprobs_amd/cli/mlprobs,
SURVEY.md section 8f row 4), generated in the build container by running
the reference pipeline's own Python stages.

The reference's utils/*.py modules are imported from /root/reference and run
in a scratch working directory laid out the way MLProbs.py expects
(./baseMSA/C_P_NP_Aln/c_p_np_aln, ./realign/QuickProbs/bin/quickprobs,
./classifier/model/*/para.txt, ./tmp/).  The two binaries there are
wrappers around the reference CLIs built from source (oracle/_ref, see
oracle/Makefile): c_p_np_aln single-threaded (taskset) with time() fixed
(oracle/fixtime.c, REF_FIXED_TIME) so -p 1 is reproducible, quickprobs with
-t 1 (its multi-threaded buildPosterior/consistency branches depend on the
schedule).  MLProbs.py itself is restated below line for line (it is a
__main__ script) with one substitution: the three RandomForest decisions
come from tests/forest_ref.py over the arrays tools/export_forests.py read
out of the reference's joblib files (the pickles cannot be loaded here;
classifier parity is checked against scikit-learn's own predict on the same
arrays, not against the 0.21.3 pickles: "parity unpinned" for that stage).

Per family the fixture holds the -G line, the classifier inputs and
decisions, the column scores, un_sp / sd / peak ratio, the regions, the
region files MLProbs wrote and realigned, and the final MSA bytes.  A second
file pins calculateColScore / getAvgColScore and both region detectors on
more MSAs (the reference's published outputs, output4evaluation/) and on
synthetic score vectors for every class_lens.

    python tests/golden/gen_pipeline.py [/root/reference]
    python tests/golden/gen_pipeline.py --heavy [workers]

--heavy writes tests/golden/pipeline_heavy/: the same per-family records for
12 TEST/ox + TEST/sabre families above 4e6 pair-cells (the families the
drop-ins send to the GPU under their default dispatch; together 46% of C5's
pair-cells), plus the reference CLIs' own outputs on each (c_p_np_aln -p 0
and -p 1 single-threaded under the fixed clock, quickprobs -t 1), one worker
process per family.
"""
import hashlib
import importlib
import json
import os
import random
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import forest_ref  # noqa: E402

HEAVY = '--heavy' in sys.argv
REF = '/root/reference' if HEAVY or len(sys.argv) < 2 else sys.argv[1]
OUT = os.path.join(HERE, 'pipeline_heavy' if HEAVY else 'pipeline')
FIXED_TIME = '1700000000'
MAX_CELLS = 4e6


def cells(path):
    lens, cur = [], None
    for line in open(path, encoding='latin-1').read().splitlines():
        if line.startswith('>'):
            if cur is not None:
                lens.append(cur)
            cur = 0
        elif cur is not None:
            cur += sum(c.isalpha() for c in line)
    if cur is not None:
        lens.append(cur)
    return sum((lens[a] + 1) * (lens[b] + 1) for a in range(len(lens)) for b in range(a + 1, len(lens)))


def setup_workdir(work, cpu=0):
    os.makedirs(os.path.join(work, 'baseMSA', 'C_P_NP_Aln'))
    os.makedirs(os.path.join(work, 'realign', 'QuickProbs', 'bin'))
    cp = os.path.join(work, 'baseMSA', 'C_P_NP_Aln', 'c_p_np_aln')
    with open(cp, 'w') as fh:
        fh.write('#!/bin/sh\nREF_FIXED_TIME=%s exec taskset -c %d %s "$@"\n'
                 % (FIXED_TIME, cpu, os.path.join(ROOT, 'oracle', '_ref', 'c_p_np_aln_ft')))
    qp = os.path.join(work, 'realign', 'QuickProbs', 'bin', 'quickprobs')
    with open(qp, 'w') as fh:
        fh.write('#!/bin/sh\nexec %s -t 1 "$@"\n' % os.path.join(ROOT, 'oracle', '_ref', 'quickprobs'))
    os.chmod(cp, 0o755)
    os.chmod(qp, 0o755)
    for m in ('branch', 'regions', 'seq_lens'):
        d = os.path.join(work, 'classifier', 'model', m)
        os.makedirs(d)
        shutil.copyfile(os.path.join(REF, 'classifier', 'model', m, 'para.txt'), os.path.join(d, 'para.txt'))


def load_reference_utils():
    sys.path.insert(0, os.path.join(REF, 'utils'))
    mods = {}
    for name in ('utils', 'prepare_features_4_classifier_1', 'classifier_c_p_np_aln', 'calculate_column_scores',
                 'unreliable_regions', 'reliable_regions', 'seperate_regions', 'do_realign'):
        mods[name] = importlib.import_module(name)
    return mods


def run_family(U, seq_file, forests):
    """MLProbs.py:36-99 with the forests' decisions from forest_ref."""
    rec = {}
    sigma, beta, threshold = 1.2, 0.0, 2.0
    realign = './realign/QuickProbs/bin/quickprobs '
    dir_output = './tmp/seperate_regions/'
    output_file = './final.msa'
    killed_stage = 0
    U['utils'].Refresh()
    rc, pid_out = subprocess.getstatusoutput('./baseMSA/C_P_NP_Aln/c_p_np_aln -G ' + seq_file)
    rec['features_line'] = pid_out
    test_list, _, avg_PID, sd_PID, factor = U['prepare_features_4_classifier_1'].getFeatures4Classifier1(seq_file)
    rec['features1'] = test_list[0]
    # testClassifier (classifier_c_p_np_aln.py:17-30)
    c = forest_ref.predict(forests['branch'], test_list[0])
    class_ = 0 if int(c) >= 2 or int(c) < 0 else int(c)
    rec['class1'] = class_
    result_real_output, killed_stage = U['classifier_c_p_np_aln'].getMSA(class_, seq_file, killed_stage)
    rec['base_msa_sha'] = hashlib.sha256(result_real_output.encode('latin-1')).hexdigest()
    _, col_score, un_sp, len_seqs, len_family, sd_un_sp, peak = \
        U['calculate_column_scores'].calculateColScore(result_real_output)
    rec.update(col_score=col_score, un_sp=un_sp, len_seqs=len_seqs, len_family=len_family, sd_un_sp=sd_un_sp,
               peak_length_ratio=peak)
    # getRealignStrategy (classifier_realign_strategy.py:13-29)
    f3 = forest_ref.normalise([peak, avg_PID, sd_un_sp, un_sp], forest_ref.load_para('regions'))
    class_region = forest_ref.predict(forests['regions'], f3)
    if class_region > 1 or class_region < 0:
        class_region = 1
    rec['class_region'] = int(class_region)
    rec['class_lens'] = -1
    if int(class_region) == 1:
        # getRegionsLength (classifier_region_min_length.py:13-29)
        f2 = forest_ref.normalise([len_seqs, len_family, avg_PID, sd_PID, un_sp], forest_ref.load_para('seq_lens'))
        class_lens = forest_ref.predict(forests['seq_lens'], f2)
        if class_lens > 3 or class_lens < 0:
            class_lens = 3
        rec['class_lens'] = int(class_lens)
        rec['regions'] = U['unreliable_regions'].getUnreliableRegions(sigma, beta, col_score, seq_file,
                                                                       result_real_output, class_lens)
        killed_stage = U['seperate_regions'].seperateCategory1Regions(seq_file, col_score, sigma, beta, class_lens,
                                                                       result_real_output, dir_output, output_file,
                                                                       killed_stage)
    else:
        rec['regions'] = U['reliable_regions'].getReliableRegions(col_score, threshold, 0, 0, seq_file, dir_output)
        killed_stage = U['seperate_regions'].seperateCategory2Regions(seq_file, col_score, threshold,
                                                                       result_real_output, dir_output, output_file,
                                                                       killed_stage)
    rec['killed_stage'] = killed_stage
    rec['region_files'] = sorted(os.listdir(dir_output))
    if killed_stage != 4:
        U['do_realign'].doRealignDir(seq_file, dir_output, realign, realign, class_region, factor)
        rec['after_realign'] = {f: open(os.path.join(dir_output, f), encoding='latin-1').read()
                                for f in sorted(os.listdir(dir_output))}
        U['do_realign'].combineFiles(seq_file, dir_output, output_file)
    else:
        if not os.path.exists(output_file) or not os.path.getsize(output_file):
            os.system(realign + ' ' + seq_file + ' > ' + output_file)
    if not os.path.getsize(output_file):
        os.system(realign + ' ' + seq_file + ' > ' + output_file)
    rec['final'] = open(output_file, encoding='latin-1').read()
    return rec


def pick_families():
    """Every 20th family of TEST/ox and TEST/sabre by name with at most
    MAX_CELLS pair-cells (the drop-ins' host path), 24 in all."""
    out = []
    for bench in ('ox', 'sabre'):
        d = os.path.join(REF, 'TEST', bench, 'in')
        names = sorted(os.listdir(d))
        picked = [n for n in names[::20] if cells(os.path.join(d, n)) <= MAX_CELLS][:12]
        out += [(bench, n, os.path.join(d, n)) for n in picked]
    return out


# the heavy set: the three largest named by the round-3 review plus the
# next-largest families of both benchmarks (4.6e6 .. 9.6e7 pair-cells)
HEAVY_FAMILIES = [('ox', '____12'), ('ox', '12t119'), ('sabre', 'sup_215'), ('ox', '12t117'), ('ox', '12t116'),
                  ('sabre', 'sup_214'), ('ox', '____22'), ('sabre', 'sup_126'), ('sabre', 'twi_114'),
                  ('ox', '___136'), ('sabre', 'sup_092'), ('sabre', 'sup_065')]


def heavy_one(job):
    """One heavy family in its own scratch working directory: the pipeline
    record plus the reference CLIs' direct outputs."""
    bench, name = job
    path = os.path.join(REF, 'TEST', bench, 'in', name)
    U = load_reference_utils()
    forests = {n: forest_ref.load_forest(n) for n in ('branch', 'regions', 'seq_lens')}
    work = tempfile.mkdtemp(prefix='mlp_heavy_')
    try:
        # one core per worker (c_p_np_aln single-threaded, as in main())
        setup_workdir(work, HEAVY_FAMILIES.index(job) % os.cpu_count())
        os.chdir(work)
        rec = run_family(U, path, forests)
        clis = {}
        for tag, cmd in (('p_0', ['./baseMSA/C_P_NP_Aln/c_p_np_aln', '-p', '0', path]),
                         ('p_1', ['./baseMSA/C_P_NP_Aln/c_p_np_aln', '-p', '1', path]),
                         ('qp', ['./realign/QuickProbs/bin/quickprobs', path])):
            r = subprocess.run(cmd, capture_output=True)
            clis[tag] = [r.returncode, r.stdout.decode('latin-1')]
        rec['reference_cli'] = clis
    finally:
        os.chdir('/')
        shutil.rmtree(work, ignore_errors=True)
    tag = f'{bench}_{name}'
    shutil.copyfile(path, os.path.join(OUT, f'{tag}.fa'))
    with open(os.path.join(OUT, f'{tag}.json'), 'w') as fh:
        json.dump(rec, fh)
    return {'family': f'{bench}/{name}', 'tag': tag, 'cells': cells(path), 'class1': rec['class1'],
            'class_region': rec['class_region'], 'class_lens': rec['class_lens'], 'regions': len(rec['regions']),
            'killed_stage': rec['killed_stage']}


def main_heavy():
    from multiprocessing import Pool
    workers = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 6
    os.makedirs(OUT, exist_ok=True)
    with Pool(workers) as pool:
        manifest = list(pool.imap(heavy_one, HEAVY_FAMILIES))
    for m in manifest:
        print(m, flush=True)
    with open(os.path.join(OUT, 'manifest.json'), 'w') as fh:
        json.dump({'generator': 'tests/golden/gen_pipeline.py --heavy',
                   'reference': 'kuangmeng/MLProbs utils/*.py + oracle/_ref CLIs (c_p_np_aln single thread, '
                                'fixed time %s; quickprobs -t 1); reference_cli: the CLIs run directly' % FIXED_TIME,
                   'families': manifest}, fh, indent=1)


def scores_fixture(U):
    """calculateColScore / getAvgColScore on published outputs, and both region
    detectors on synthetic score vectors."""
    rnd = random.Random(7)
    msas = []
    for bench in ('ox', 'sabre', 'bali3'):
        d = os.path.join(REF, 'output4evaluation', bench)
        names = sorted(os.listdir(d))[::40][:6]
        for n in names:
            text = open(os.path.join(d, n), encoding='latin-1').read()
            # as subprocess.getstatusoutput hands it over: one trailing newline removed
            _, col, un, L, N, sd, peak = U['calculate_column_scores'].calculateColScore(
                text[:-1] if text.endswith('\n') else text)
            path = os.path.join(tempfile.gettempdir(), 'mlp_avg.msa')
            with open(path, 'w', encoding='latin-1') as fh:
                fh.write(text)
            avg = U['calculate_column_scores'].getAvgColScore(path)
            msas.append({'name': f'{bench}/{n}', 'text': text, 'col_score': col, 'un_sp': un, 'len_seqs': L,
                         'len_family': N, 'sd_un_sp': sd, 'peak_length_ratio': peak, 'avg_col_score': avg})
    regions = []
    for k in range(60):
        L = rnd.randint(1, 400)
        col = [rnd.choice([rnd.uniform(-2, 3), rnd.uniform(0, 1.2), rnd.uniform(1.5, 6), 0.0, 1.2, 2.0])
               for _ in range(L)]
        rec = {'col_score': col, 'unreliable': {}, 'reliable': None}
        for cl in (0, 1, 2, 3):
            rec['unreliable'][str(cl)] = U['unreliable_regions'].getUnreliableRegions(1.2, 0.0, col, '', '', cl)
        rec['reliable'] = U['reliable_regions'].getReliableRegions(col, 2.0, 0, 0, '', '')
        regions.append(rec)
    return {'msas': msas, 'regions': regions}


def main():
    U = load_reference_utils()
    forests = {n: forest_ref.load_forest(n) for n in ('branch', 'regions', 'seq_lens')}
    os.makedirs(OUT, exist_ok=True)
    manifest = []
    cwd = os.getcwd()
    work = tempfile.mkdtemp(prefix='mlp_pipe_')
    try:
        setup_workdir(work)
        os.chdir(work)
        for bench, name, path in pick_families():
            rec = run_family(U, path, forests)
            tag = f'{bench}_{name}'
            shutil.copyfile(path, os.path.join(OUT, f'{tag}.fa'))
            with open(os.path.join(OUT, f'{tag}.json'), 'w') as fh:
                json.dump(rec, fh)
            manifest.append({'family': f'{bench}/{name}', 'tag': tag, 'class1': rec['class1'],
                             'class_region': rec['class_region'], 'class_lens': rec['class_lens'],
                             'regions': len(rec['regions']), 'killed_stage': rec['killed_stage']})
            print(manifest[-1], flush=True)
        with open(os.path.join(OUT, 'scores.json'), 'w') as fh:
            json.dump(scores_fixture(U), fh)
    finally:
        os.chdir(cwd)
        shutil.rmtree(work, ignore_errors=True)
    with open(os.path.join(OUT, 'manifest.json'), 'w') as fh:
        json.dump({'generator': 'tests/golden/gen_pipeline.py', 'reference': 'kuangmeng/MLProbs utils/*.py + '
                   'oracle/_ref CLIs (c_p_np_aln single thread, fixed time %s; quickprobs -t 1)' % FIXED_TIME,
                   'families': manifest}, fh, indent=1)


if __name__ == '__main__':
    main_heavy() if HEAVY else main()
