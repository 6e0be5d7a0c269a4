"""Dev tool (round 5 hygiene): resolve compile-time A/B knobs in a source file.

  python tools/unknob.py <file> NAME=value [NAME=value ...]

For each NAME: the `#ifndef NAME / #define NAME v / #endif` default block is dropped, `#if` / `#elif`
conditions that are exactly `NAME`, `!NAME`, `NAME == k`, `NAME != k` (or their `defined` forms) are
evaluated with the given value and their dead branches removed, and remaining uses of NAME in code are
replaced by the value.  Conditions mentioning other macros are left alone (the tool refuses a condition
that mixes a resolved NAME with anything else).
"""
import re
import sys


def cond_value(cond, vals):
    c = cond.strip()
    c = re.sub(r'//.*$', '', c).strip()
    m = re.fullmatch(r'(!?)\s*(\w+)', c)
    if m and m.group(2) in vals:
        v = bool(int(vals[m.group(2)]))
        return (not v) if m.group(1) else v
    m = re.fullmatch(r'(\w+)\s*(==|!=)\s*(-?\d+)', c)
    if m and m.group(1) in vals:
        eq = int(vals[m.group(1)]) == int(m.group(3))
        return eq if m.group(2) == '==' else not eq
    for n in vals:
        if re.search(r'\b%s\b' % n, c):
            raise SystemExit(f'condition mixes {n} with other terms: {cond!r}')
    return None


def main():
    path = sys.argv[1]
    vals = dict(a.split('=', 1) for a in sys.argv[2:])
    lines = open(path).read().split('\n')
    out = []
    # stack entries: [resolved (bool|None), keep_current (bool), any_taken (bool), parent_keep]
    stack = []
    keep = True
    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        m = re.match(r'#\s*ifndef\s+(\w+)\s*$', s)
        if m and m.group(1) in vals and i + 2 < len(lines) and \
                re.match(r'#\s*define\s+%s\b' % m.group(1), lines[i + 1].strip()) and \
                lines[i + 2].strip().startswith('#endif'):
            i += 3   # the default definition
            continue
        m = re.match(r'#\s*if\s+(.*)$', s)
        if m and not s.startswith('#ifdef') and not s.startswith('#ifndef'):
            r = cond_value(m.group(1), vals)
            stack.append([r, keep, r is True])
            if r is None:
                if keep:
                    out.append(ln)
            else:
                keep = keep and r
            i += 1
            continue
        if re.match(r'#\s*if(n?def)\b', s):
            stack.append([None, keep, False])
            if keep:
                out.append(ln)
            i += 1
            continue
        m = re.match(r'#\s*elif\s+(.*)$', s)
        if m:
            top = stack[-1]
            if top[0] is None:
                if top[1]:
                    out.append(ln)
            else:
                r = cond_value(m.group(1), vals)
                if r is None:
                    raise SystemExit(f'#elif with unresolved condition after a resolved #if: {s}')
                take = r and not top[2]
                top[2] = top[2] or take
                keep = top[1] and take
            i += 1
            continue
        if re.match(r'#\s*else\b', s):
            top = stack[-1]
            if top[0] is None:
                if top[1]:
                    out.append(ln)
            else:
                keep = top[1] and not top[2]
                top[2] = True
            i += 1
            continue
        if re.match(r'#\s*endif\b', s):
            top = stack.pop()
            if top[0] is None:
                if top[1]:
                    out.append(ln)
            keep = top[1]
            i += 1
            continue
        if keep:
            for n, v in vals.items():
                ln = re.sub(r'\b%s\b' % n, v, ln)
            out.append(ln)
        i += 1
    assert not stack, 'unbalanced #if'
    open(path, 'w').write('\n'.join(out))


if __name__ == '__main__':
    main()
