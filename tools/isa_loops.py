"""List the loops of each kernel in a gfx950 .s file (from hipcc --save-temps)
with their instruction counts and VMEM wait instructions, to spot
per-step s_waitcnt vmcnt drains in the DP step loops.

    python tools/isa_loops.py posterior-hip-amdgcn-amd-amdhsa-gfx950.s [name-filter]
"""
import re
import sys


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    lines = open(path).read().splitlines()
    fn = None
    body = []
    funcs = []
    for ln in lines:
        m = re.match(r'^(_Z\w+):', ln)
        if m:
            fn = m.group(1)
            body = []
            funcs.append((fn, body))
            continue
        if fn is not None:
            if ln.strip().startswith('.Lfunc_end'):
                fn = None
                continue
            body.append(ln)
    for fn, body in funcs:
        if filt not in fn:
            continue
        labels = {}
        for k, ln in enumerate(body):
            m = re.match(r'^(\.LBB\w+):', ln)
            if m:
                labels[m.group(1)] = k
        print(fn)
        for k, ln in enumerate(body):
            m = re.match(r'\s+s_(?:c)?branch\w*\s+(\.LBB\w+)', ln)
            if m and m.group(1) in labels and labels[m.group(1)] < k:
                a = labels[m.group(1)]
                seg = body[a:k + 1]
                ins = [x for x in seg if x.startswith('\t') and not x.strip().startswith(('.', ';'))]
                waits = [x.strip() for x in seg if 's_waitcnt' in x and 'vmcnt' in x]
                nload = sum(1 for x in seg if 'global_load' in x or 'buffer_load' in x)
                nstore = sum(1 for x in seg if 'global_store' in x or 'buffer_store' in x)
                print(f'  loop {m.group(1)} lines {a}-{k}: {len(ins)} instr, {nload} loads, {nstore} stores, '
                      f'{len(waits)} vm waits: {sorted(set(waits))[:6]}')


if __name__ == '__main__':
    main()
