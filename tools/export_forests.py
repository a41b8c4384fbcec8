"""Export MLProbs' three RandomForest classifiers (classifier/model/{branch,
regions,seq_lens}/randomforest.joblib, scikit-learn 0.21.3 pickles written by
joblib 0.13) as plain arrays for the pipeline driver's own forest evaluator.

Nothing in the files is executed.  `pickle`/`joblib` are never called: the
opcode stream is read with `pickletools.genops` (a disassembler) and
interpreted here into inert values -- globals become ('global', module,
name) tags, REDUCE / NEWOBJ become ('call', tag, args) records whose BUILD
state is attached as data.  Only the handful of record shapes a forest uses
are then turned into numpy arrays by this script's own code:
  * numpy.dtype(...) + its state tuple          -> np.dtype
  * joblib NumpyArrayWrapper + the raw bytes that follow its BUILD in the
    file (joblib 0.13 writes no alignment padding)   -> np.ndarray
  * sklearn.tree._tree.Tree(n_features, n_classes, n_outputs) + state dict
    {'nodes', 'values', ...}                      -> the tree's arrays
Anything else stays an inert record and is ignored.

Output (mlprobs_amd/classifier/<name>.forest, little endian):
  b'MLPF', u32 version 1, u32 n_trees, u32 n_features, u32 n_classes,
  f64 classes[n_classes], then per tree: u32 node_count, i32 left[nc],
  i32 right[nc], i32 feature[nc], f64 threshold[nc], f64 value[nc * n_classes]
(leaf: left = -1; value = the weighted class counts sklearn keeps), plus
<name>.para (the reference's min-max normalisation file, copied).

    python tools/export_forests.py [/root/reference]
"""
import os
import pickletools
import shutil
import struct
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'mlprobs_amd', 'classifier')
NAMES = ('branch', 'regions', 'seq_lens')


class Rec:
    """An inert record: a global reference called with args, plus state."""

    def __init__(self, func, args):
        self.func, self.args, self.state = func, args, None
        self.items = None   # list/dict contents when used as a container target


def _dtype(rec):
    """numpy.dtype(spec, align, copy) with its __setstate__ tuple."""
    spec = rec.args[0]
    st = rec.state
    order = st[1] if st else '|'
    names, fields = (st[3], st[4]) if st else (None, None)
    if names:
        formats, offsets = [], []
        for n in names:
            sub = fields[n][0]
            formats.append(_dtype(sub) if isinstance(sub, Rec) else sub)
            offsets.append(fields[n][1])
        return np.dtype({'names': list(names), 'formats': formats, 'offsets': offsets, 'itemsize': st[5]})
    dt = np.dtype(spec)
    if order in '<>':
        dt = dt.newbyteorder(order)
    return dt


def read_joblib(path):
    """Interpret the pickle stream of a joblib file into inert values."""
    f = open(path, 'rb')
    stack, marks, memo = [], [], {}

    def pop_mark():
        k = marks.pop()
        items = stack[k:]
        del stack[k:]
        return items

    ops = pickletools.genops(f)
    for op, arg, _pos in ops:
        name = op.name
        if name == 'PROTO':
            continue
        if name == 'STOP':
            break
        if name in ('GLOBAL', 'STACK_GLOBAL'):
            if name == 'GLOBAL':
                mod, nm = arg.split(' ', 1)
            else:
                nm, mod = stack.pop(), stack.pop()
            stack.append(('global', mod, nm))
        elif name == 'MARK':
            marks.append(len(stack))
        elif name in ('BINPUT', 'LONG_BINPUT', 'PUT'):
            memo[arg] = stack[-1]
        elif name == 'MEMOIZE':
            memo[len(memo)] = stack[-1]
        elif name in ('BINGET', 'LONG_BINGET', 'GET'):
            stack.append(memo[arg])
        elif name in ('BINUNICODE', 'SHORT_BINUNICODE', 'BINUNICODE8', 'UNICODE', 'BININT', 'BININT1', 'BININT2',
                      'LONG1', 'LONG4', 'BINFLOAT', 'BINSTRING', 'SHORT_BINSTRING', 'BINBYTES', 'SHORT_BINBYTES',
                      'BINBYTES8', 'INT', 'LONG', 'FLOAT', 'STRING'):
            stack.append(arg)
        elif name == 'NONE':
            stack.append(None)
        elif name == 'NEWTRUE':
            stack.append(True)
        elif name == 'NEWFALSE':
            stack.append(False)
        elif name == 'EMPTY_DICT':
            stack.append({})
        elif name == 'EMPTY_LIST':
            stack.append([])
        elif name == 'EMPTY_TUPLE':
            stack.append(())
        elif name == 'TUPLE':
            stack.append(tuple(pop_mark()))
        elif name in ('TUPLE1', 'TUPLE2', 'TUPLE3'):
            k = int(name[-1])
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif name == 'LIST':
            stack.append(list(pop_mark()))
        elif name == 'DICT':
            it = pop_mark()
            stack.append({it[i]: it[i + 1] for i in range(0, len(it), 2)})
        elif name == 'APPEND':
            v = stack.pop()
            stack[-1].append(v)
        elif name == 'APPENDS':
            it = pop_mark()
            stack[-1].extend(it)
        elif name == 'SETITEM':
            v, k = stack.pop(), stack.pop()
            stack[-1][k] = v
        elif name == 'SETITEMS':
            it = pop_mark()
            for i in range(0, len(it), 2):
                stack[-1][it[i]] = it[i + 1]
        elif name in ('REDUCE', 'NEWOBJ'):
            args, func = stack.pop(), stack.pop()
            stack.append(Rec(func, args))
        elif name == 'BUILD':
            state = stack.pop()
            obj = stack[-1]
            if not isinstance(obj, Rec):
                raise ValueError(f'BUILD on {type(obj)}')
            obj.state = state
            if obj.func == ('global', 'joblib.numpy_pickle', 'NumpyArrayWrapper'):
                dt = _dtype(state['dtype'])
                if dt.hasobject:
                    raise ValueError('object arrays are not read')
                shape = tuple(state['shape'])
                count = int(np.prod(shape)) if shape else 1
                raw = f.read(count * dt.itemsize)   # the array bytes follow the BUILD
                arr = np.frombuffer(raw, dtype=dt, count=count).reshape(shape, order=state['order'])
                stack[-1] = arr.copy()
        elif name == 'POP':
            stack.pop()
        elif name == 'POP_MARK':
            pop_mark()
        elif name == 'DUP':
            stack.append(stack[-1])
        else:
            raise ValueError(f'unhandled opcode {name}')
    f.close()
    return stack[-1]


def forest_arrays(top):
    """(classes, n_features, [(left, right, feature, threshold, value)]) of the
    RandomForestClassifier record `top`."""
    if top.func != ('global', 'sklearn.ensemble.forest', 'RandomForestClassifier'):
        raise ValueError(f'unexpected top-level record {top.func}')
    st = top.state
    classes = np.asarray(st['classes_'], np.float64)
    trees = []
    for est in st['estimators_']:
        tree = est.state['tree_']
        if tree.func != ('global', 'sklearn.tree._tree', 'Tree'):
            raise ValueError(f'unexpected tree record {tree.func}')
        ts = tree.state
        nodes, values = ts['nodes'], ts['values']
        nc = int(ts['node_count'])
        assert nodes.shape[0] == nc and values.shape[0] == nc and values.shape[1] == 1
        trees.append((nodes['left_child'].astype(np.int32), nodes['right_child'].astype(np.int32),
                      nodes['feature'].astype(np.int32), nodes['threshold'].astype(np.float64),
                      values[:, 0, :].astype(np.float64)))
    return classes, int(st['n_features_']), trees


def write_forest(path, classes, n_features, trees):
    with open(path, 'wb') as fh:
        fh.write(b'MLPF' + struct.pack('<4I', 1, len(trees), n_features, len(classes)))
        fh.write(classes.astype('<f8').tobytes())
        for left, right, feat, thr, val in trees:
            fh.write(struct.pack('<I', len(left)))
            for a, dt in ((left, '<i4'), (right, '<i4'), (feat, '<i4'), (thr, '<f8'), (val, '<f8')):
                fh.write(np.ascontiguousarray(a, dt).tobytes())


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else '/root/reference'
    os.makedirs(OUT, exist_ok=True)
    for name in NAMES:
        d = os.path.join(ref, 'classifier', 'model', name)
        top = read_joblib(os.path.join(d, 'randomforest.joblib'))
        classes, nf, trees = forest_arrays(top)
        write_forest(os.path.join(OUT, f'{name}.forest'), classes, nf, trees)
        shutil.copyfile(os.path.join(d, 'para.txt'), os.path.join(OUT, f'{name}.para'))
        print(f'{name}: {len(trees)} trees, {nf} features, classes {classes.tolist()}, '
              f'{sum(len(t[0]) for t in trees)} nodes')


if __name__ == '__main__':
    main()
