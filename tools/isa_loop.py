"""Instruction counts of the FABRIK iteration kernel's inner loop (the CORE 2
step), from a device assembly file (hipcc --cuda-device-only -S ik_fabrik.hip):
each basic-block segment between the loop header that runs the step and the
back edge, with its VALU / fp64 / SALU counts.  Development aid.

    python tools/isa_loop.py fab.s [kernel-substring]

(With -DIKHIP_PHASE_MARKS the loop is the first inner loop after ';@phase loop';
without, the inner loop with the most v_rsq_f64, which since r06 can be the retire
step's re-solve loop.)
"""
import re
import sys


def segments(path, kern):
    s = open(path).read()
    k = s.index(kern)
    k = s.index(':', k)
    e = s.index('.Lfunc_end', k)
    segs = []
    for line in s[k:e].split('\n'):
        m = re.match(r'^(\.LBB\S+):(.*)$', line)
        m2 = re.match(r'^; %bb\.(\d+):(.*)$', line)
        if m:
            segs.append([m.group(1), m.group(2), []])
        elif m2:
            segs.append(['%bb.' + m2.group(1), m2.group(2), []])
        elif segs and line.startswith('\t') and not line.startswith('\t.') and not line.startswith('\t;'):
            segs[-1][2].append(line.strip())
        elif segs and line.strip().startswith(';') and 'Loop' in line:
            segs[-1][1] += line
    return segs


def main():
    path = sys.argv[1]
    kern = sys.argv[2] if len(sys.argv) > 2 else '_ZN5ikhip18fabrik_iter_kernelILi12ELb1ELi2EEEvNS_7FabArgsE'
    segs = segments(path, kern)
    hdrs = [i for i, sg in enumerate(segs) if 'Inner Loop Header' in sg[1] and 'Depth=2' in sg[1]]
    best = None
    text = open(path).read()
    if ';@phase loop' in text:
        # a -DIKHIP_PHASE_MARKS build: the first inner loop after the kernel's
        # ';@phase loop' mark is the iteration loop (the flush's re-solve loop,
        # solve_general, holds more v_rsq_f64 than it)
        rest = text[text.index(';@phase loop', text.index(kern + ':')):]
        j = rest.index('This Inner Loop Header')
        line_start = rest.rfind('\n', 0, j)
        hdr_name = rest[rest.rfind('\n', 0, line_start) + 1:j].split(':')[0].strip()
        for h in hdrs:
            if segs[h][0] == hdr_name:
                name = segs[h][0].split('_')[-1]
                body = [i for i, sg in enumerate(segs)
                        if i == h or f'Header=BB{segs[h][0][4:].split("_")[0]}_{name} ' in sg[1] + ' ']
                best = (sum(sum('v_rsq_f64' in x for x in segs[i][2]) for i in body), body)
    for h in hdrs if best is None else []:
        # without marks: the inner loop holding the most v_rsq_f64
        name = segs[h][0].split('_')[-1]
        body = [i for i, sg in enumerate(segs)
                if i == h or f'Header=BB{segs[h][0][4:].split("_")[0]}_{name} ' in sg[1] + ' ']
        rsq = sum(sum('v_rsq_f64' in x for x in segs[i][2]) for i in body)
        if best is None or rsq > best[0]:
            best = (rsq, body)
    tot = [0, 0, 0]
    for i in best[1]:
        n, _, b = segs[i]
        v = sum(x.startswith('v_') for x in b)
        f = sum('f64' in x for x in b)
        sa = sum(x.startswith('s_') for x in b)
        br = [x for x in b if 'branch' in x]
        print(f'{n:12s} n={len(b):4d} valu={v:4d} f64={f:4d} salu={sa:3d} {br}')
    print('rsq in loop:', best[0])


if __name__ == '__main__':
    main()
