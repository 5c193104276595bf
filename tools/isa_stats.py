"""Instruction statistics of one kernel in a device assembly listing (make asm -> /tmp/qdc_f32.s).
usage: python3 tools/isa_stats.py <asm> <mangled-name-prefix> [--blocks]"""
import collections
import sys


def kernel_lines(path, prefix):
    S = open(path).read().split('\n')
    start = next(i for i, l in enumerate(S) if l.startswith(prefix) and l.split(':')[0].endswith('m'))
    end = next(i for i in range(start + 10, len(S)) if S[i].startswith('_Z') and ':' in S[i])
    out = []
    for l in S[start:end]:
        t = l.strip()
        if not t or t.startswith((';', '.file', '.p2align', '.loc', '.cfi')):
            continue
        out.append(t)
    return out


def main():
    L = kernel_lines(sys.argv[1], sys.argv[2])
    c = collections.Counter()
    blocks, cur = [], ['entry', collections.Counter()]
    blocks.append(cur)
    for t in L:
        if t.split()[0].endswith(':'):
            cur = [t.split()[0], collections.Counter()]
            blocks.append(cur)
            continue
        if t.startswith('.'):
            continue
        op = t.split()[0]
        c[op] += 1
        cur[1][op] += 1
        if op.startswith('scratch'):
            cur[1]['SCR:' + t.split(';')[0].strip()] += 1
    print('total', sum(v for k, v in c.items()), {k: c[k] for k in (
        'v_pk_fma_f32', 'v_pk_mul_f32', 's_nop', 's_waitcnt', 'ds_add_f32', 'ds_read_b32',
        'scratch_store_dwordx2', 'scratch_load_dwordx2', 'v_writelane_b32', 'v_readlane_b32',
        's_load_dwordx16', 'v_permlane32_swap_b32_e32', 'v_permlane16_swap_b32_e32')})
    if '--blocks' in sys.argv:
        for name, bc in blocks:
            if bc['v_pk_fma_f32'] > 60:
                scr = {k: v for k, v in bc.items() if k.startswith('SCR:')}
                print(name, sum(v for k, v in bc.items() if not k.startswith('SCR:')), 'fma', bc['v_pk_fma_f32'],
                      'wait', bc['s_waitcnt'], 'nop', bc['s_nop'], scr)


if __name__ == '__main__':
    main()
