"""Instruction counts of the FABRIK iteration kernel's inner loop (the CORE 2
step), from a device assembly file (hipcc --cuda-device-only -S ik_fabrik.hip):
each basic-block segment between the loop header that runs the step and the
back edge, with its VALU / fp64 / SALU counts.  Development aid.

    python tools/isa_loop.py fab.s [kernel-substring]
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
    kern = sys.argv[2] if len(sys.argv) > 2 else '_ZN5ikhip18fabrik_iter_kernelILi8ELb1ELi2EEEvNS_7FabArgsE'
    segs = segments(path, kern)
    # the inner loop holding the most v_rsq_f64: its header's segments in order
    hdrs = [i for i, sg in enumerate(segs) if 'Inner Loop Header' in sg[1] and 'Depth=2' in sg[1]]
    best = None
    for h in hdrs:
        name = segs[h][0].split('_')[-1]
        body = [i for i, sg in enumerate(segs) if i == h or f'Header=BB12_{name} ' in sg[1] + ' ']
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
