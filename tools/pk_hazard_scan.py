"""Static scan of packed-FP32 VALU instructions in a gfx950 assembly listing (dev tool).

For every v_pk_{fma,mul,add,mov}_f32 / v_pk_mov_b32 it finds the nearest earlier instruction (same
basic block, up to 8 instructions back) writing one of its source VGPRs and classifies that producer:
  trans     v_exp / v_log / v_rcp / v_rsq / v_sqrt / v_sin / v_cos (gfx950: trans -> VALU forwarding
            needs a wait state)
  sdwa/opsel a partial-dword write (SDWA dst_sel other than DWORD, or op_sel dst) -- gfx940+ needs a
            wait state before a VALU reads it
  mfma      an MFMA result (VALU read of an MFMA destination needs several wait states)
  lds/vmem  a load (covered by s_waitcnt)
  valu      any other VALU write
and prints, per class, how many packed instructions read such a producer with fewer than the needed
wait states between them (s_nop N counts N + 1).  Usage:
  python tools/pk_hazard_scan.py file.s [kernel-symbol-substring]
"""
import re
import sys

TRANS = ('v_exp_', 'v_log_', 'v_rcp_', 'v_rsq_', 'v_sqrt_', 'v_sin_', 'v_cos_')
NEED = {'trans': 1, 'sdwa/opsel': 1, 'mfma': 4}


def regs(tok):
    """VGPR numbers named by one operand token (v5, v[4:7])"""
    m = re.match(r'-?\|?v\[(\d+):(\d+)\]', tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r'-?\|?v(\d+)\b', tok)
    return {int(m.group(1))} if m else set()


def parse(line):
    t = line.strip()
    if not t or t.startswith(('.', ';')) or t.endswith(':'):
        return None
    t = t.split(';')[0].strip()
    op, _, rest = t.partition(' ')
    ops = [o.strip() for o in re.split(r',\s*', rest)] if rest else []
    return op, ops, t


def kind(op, text):
    if op.startswith(TRANS):
        return 'trans'
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global_', 'buffer_', 'flat_', 'scratch_')):
        return 'vmem'
    if 'dst_sel:' in text and 'dst_sel:DWORD' not in text:
        return 'sdwa/opsel'
    if op.startswith('v_'):
        return 'valu'
    return None


def scan(lines):
    out = {}
    window = []          # (op, dst regs, kind, wait states before it)
    for line in lines:
        if re.match(r'^\.LBB|^_Z', line):
            window = []
            continue
        p = parse(line)
        if p is None:
            continue
        op, ops, text = p
        if op == 's_nop':
            n = int(ops[0], 0) + 1 if ops else 1
            window = [(o, d, k, w + n) for o, d, k, w in window]
            continue
        if op.startswith('v_pk_') and (op.endswith('_f32') or op == 'v_pk_mov_b32'):
            src = set()
            for tok in ops[1:]:
                src |= regs(tok)
            for o, d, k, w in reversed(window):
                if d & src:
                    short = k in NEED and w < NEED[k]
                    key = (k, 'SHORT' if short else 'ok')
                    out.setdefault(key, []).append(f'{o} -> {text}')
                    break
        k = kind(op, text)
        if k is None:      # SALU, waits, branches: one wait state each, no VGPR written
            window = [(o, d, kk, w + 1) for o, d, kk, w in window]
            continue
        dst = set()
        if ops and (k not in ('lds', 'vmem') or op.startswith(('ds_read', 'global_load', 'buffer_load', 'scratch_load', 'ds_bpermute'))):
            dst = regs(ops[0])
        window = [(o, d, kk, w + 1) for o, d, kk, w in window][-7:] + [(op, dst, k, 0)]
    return out


def swaps(lines):
    """packed instructions whose low lane reads a source's high dword (op_sel bit set), split into
    broadcasts (that source's op_sel_hi bit also set) and half-swaps (op_sel_hi bit clear)"""
    bc = sw = 0
    for l in lines:
        m = re.match(r'\s*(v_pk_\w+)\s+(.*)', l)
        if not m or not (m.group(1).endswith('_f32') or m.group(1) == 'v_pk_mov_b32'):
            continue
        nsrc = 2 if m.group(1) == 'v_pk_mov_b32' or not m.group(1).startswith('v_pk_fma') else 3
        os_ = re.search(r'op_sel:\[([\d,]+)\]', m.group(2))
        oh = re.search(r'op_sel_hi:\[([\d,]+)\]', m.group(2))
        lo = [int(x) for x in os_.group(1).split(',')] if os_ else [0] * nsrc
        hi = [int(x) for x in oh.group(1).split(',')] if oh else [1] * nsrc
        for a, b in zip(lo, hi):
            if a:
                if b:
                    bc += 1
                else:
                    sw += 1
    return bc, sw


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else None
    lines = open(path).read().split('\n')
    if want:
        starts = [i for i, l in enumerate(lines) if re.match(r'^_Z\S*:', l)]
        sel = []
        for j, i in enumerate(starts):
            if want in lines[i]:
                end = starts[j + 1] if j + 1 < len(starts) else len(lines)
                sel += lines[i:end]
        lines = sel
    res = scan(lines)
    n_pk = sum(1 for l in lines if re.match(r'\s*v_pk_\w+_f32|\s*v_pk_mov_b32', l))
    bc, sw = swaps(lines)
    print(f'{n_pk} packed-FP32 instructions; low lane reading a high dword: {bc} broadcast, {sw} half-swapped operands')
    for (k, s), v in sorted(res.items()):
        print(f'  producer {k:10s} {s:5s} {len(v):5d}' + (f'   e.g. {v[0]}' if s == 'SHORT' else ''))


if __name__ == '__main__':
    main()
