"""Instructions per lean stage in a kernel's ISA: the distance between
consecutive v_rsq_f64 (one per stage, the corner distance of local_collide)
inside the unrolled 20-stage loop, split into VALU / SALU / other, plus the
DPP moves and waits.  usage: isa_stage_count.py <file.s> <kernel-substring>"""
import re
import sys


def kernel_body(path, name):
    lines = open(path).read().splitlines()
    start = None
    for i, ln in enumerate(lines):
        if start is None and re.match(r'^\S*' + re.escape(name) + r'\S*:\s*(;.*)?$', ln) and '.L' not in ln[:2]:
            start = i
        elif start is not None and ln.startswith('.Lfunc_end'):
            return lines[start:i]
    raise SystemExit(f'kernel {name} not found')


def main():
    body = kernel_body(sys.argv[1], sys.argv[2])
    ins = [ln.strip() for ln in body if ln.startswith('\t') and not ln.strip().startswith(('.', ';'))]
    rsq = [i for i, s in enumerate(ins) if s.startswith('v_rsq_f64')]
    gaps = [b - a for a, b in zip(rsq, rsq[1:])]
    steady = gaps[1:-1] if len(gaps) > 2 else gaps
    seg = ins[rsq[1]:rsq[-2]] if len(rsq) > 3 else ins
    n = max(1, len(steady))
    kinds = dict(valu=sum(s.startswith('v_') for s in seg) / n, salu=sum(s.startswith('s_') and not s.startswith(('s_nop', 's_waitcnt')) for s in seg) / n,
                 dpp=sum('quad_perm' in s or 'row_' in s for s in seg) / n, nop=sum(s.startswith('s_nop') for s in seg) / n,
                 cndmask=sum(s.startswith('v_cndmask') for s in seg) / n)
    print(f'{sys.argv[2]}: {len(ins)} instructions, {len(rsq)} v_rsq_f64; steady stage gaps {steady}; '
          f'mean {sum(steady) / n:.1f} per stage; per stage ' + ', '.join(f'{k} {v:.1f}' for k, v in kinds.items()))


if __name__ == '__main__':
    main()
