import itertools
G128 = [list(range(0,4))+list(range(12,16))+list(range(20,28)), list(range(4,12))+list(range(16,20))+list(range(28,32))]
G128 = G128 + [[l+32 for l in g] for g in G128]
def cycles_b128(addrs):
    tot = 0
    for g in G128:
        banks = {}
        for l in g:
            a = addrs[l]
            for d in range(4):
                b = (a // 4 + d) % 64
                banks.setdefault(b, set()).add(a // 16)
        tot += max(len(v) for v in banks.values())
    return tot  # ideal 4
def conv_reads(TW, KH, KW, LDP, swz=None):
    WP = TW + KW - 1
    tot = 0; cnt = 0
    for dy in range(KH):
        for dx in range(KW):
            for s in range(2):  # CK=32 -> 2 ksteps of 16
                for mbase in (0, 32, 64, 96):
                    addrs = []
                    for lane in range(64):
                        m = mbase + (lane & 31)
                        pix = (m // TW + dy) * WP + (m % TW + dx)
                        chunk = 2 * s + (lane >> 5)      # 16-B chunk of the 64-B pixel data
                        if swz: chunk = swz(pix, chunk)
                        addrs.append(pix * LDP * 2 + chunk * 16)
                    tot += cycles_b128(addrs); cnt += 1
    return tot / cnt
for TW, KH, KW in ((8,3,3),(8,4,1),(16,3,3),(16,4,1),(1,3,1)):
    print(TW, KH, KW, 'LDP40', conv_reads(TW,KH,KW,40), 'LDP32', conv_reads(TW,KH,KW,32), 'LDP48', conv_reads(TW,KH,KW,48),
          'LDP32 xor', conv_reads(TW,KH,KW,32, lambda p,c: c ^ ((p >> 1) & 3)), 'LDP32 xor2', conv_reads(TW,KH,KW,32, lambda p,c: c ^ (p & 3)))
print('---search')
def conv_reads2(TW, KH, KW, LDP, WPP, swz):
    WP = TW + KW - 1
    tot = 0; cnt = 0
    for dy in range(KH):
        for dx in range(KW):
            for s in range(2):
                for mbase in (0, 32, 64, 96):
                    addrs = []
                    for lane in range(64):
                        m = mbase + (lane & 31)
                        r, c = m // TW + dy, m % TW + dx
                        pix = r * WPP + c
                        chunk = 2 * s + (lane >> 5)
                        chunk = swz(r, c, pix, chunk)
                        addrs.append(pix * LDP * 2 + chunk * 16)
                    tot += cycles_b128(addrs); cnt += 1
    return tot / cnt
swzs = {'none': lambda r,c,p,ch: ch,
        'r&3': lambda r,c,p,ch: ch ^ (r & 3), 'r>>1&3': lambda r,c,p,ch: ch ^ ((r>>1)&3),
        'c>>1&3': lambda r,c,p,ch: ch ^ ((c>>1)&3), 'c>>2&3': lambda r,c,p,ch: ch ^ ((c>>2)&3),
        'c>>3&3': lambda r,c,p,ch: ch ^ ((c>>3)&3), '(r^c>>2)&3': lambda r,c,p,ch: ch ^ ((r ^ (c>>2))&3),
        'r&1<<1': lambda r,c,p,ch: ch ^ ((r&1)<<1), '(c>>3)+2r': lambda r,c,p,ch: ch ^ (((c>>3) + 2*r)&3)}
best = {}
for TW, KH, KW in ((8,3,3),(16,3,3),(8,4,1),(16,4,1),(1,3,1)):
    WP = TW + KW - 1
    res = []
    for LDP in (40, 48, 56):
        for WPP in sorted(set([WP, WP+1, WP+2, WP+6, 12, 16, 20])):
            if WPP < WP: continue
            for name, f in swzs.items():
                cyc = conv_reads2(TW,KH,KW,LDP,WPP,f)
                res.append((cyc, LDP*WPP, LDP, WPP, name))
    res.sort()
    print(TW,KH,KW, res[:6])
print('---search2')
for TW, KH, KW in ((8,3,3),(16,3,3)):
    WP = TW + KW - 1
    res = []
    for LDP in (40, 48):
        nch = LDP // 8
        for WPP in range(WP, WP + 7):
            for a in range(5):
                for b in range(4):
                    for g in range(5):
                        for mode in ('xor', 'rot'):
                            if mode == 'xor':
                                f = lambda r,c,p,ch,a=a,b=b,g=g: ch ^ ((a*r + g*(c>>b)) & 3)
                            else:
                                f = lambda r,c,p,ch,a=a,b=b,g=g,n=nch: (ch + a*r + g*(c>>b)) % n
                            cyc = conv_reads2(TW,KH,KW,LDP,WPP,f)
                            res.append((cyc, LDP*WPP, LDP, WPP, mode, a, b, g))
    res.sort()
    print(TW,KH,KW, res[:8])
