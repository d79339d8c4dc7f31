# CPU restatement of k_snappy.hip's chunk speculation, entry rules and region resolver (spec /
# assume / entries / regions / resolve), used to find and check the r02 resolver fix: run
# resolve_all(pyarrow.compress(data, "snappy", asbytes=True)) with FIX = False / True.
FIX = True  # the r02 stop rule (False: the earlier one)
"""CPU simulation of k_snappy.hip's chunk speculation + entry rules (spec/assume/entries) to find
chunks whose entries are wrong without being flagged."""
import sys
import numpy as np
import pyarrow as pa

def elem(b, pos):
    tag = b[pos]; t = tag & 3
    if t == 0:
        l6 = tag >> 2
        if l6 < 60: return 1 + l6 + 1, l6 + 1, 0
        nb = l6 - 59; v = int.from_bytes(bytes(b[pos+1:pos+1+nb]), 'little')
        return 1 + nb + v + 1, v + 1, 0
    if t == 1: return 2, ((tag >> 2) & 7) + 4, ((tag >> 5) << 8) | b[pos+1]
    if t == 2: return 3, (tag >> 2) + 1, b[pos+1] | (b[pos+2] << 8)
    return 5, (tag >> 2) + 1, int.from_bytes(bytes(b[pos+1:pos+5]), 'little')

def run(raw, CH=256, WU=192, MAX_RUN=32):
    # strip preamble
    pre = 0
    while raw[pre] & 0x80: pre += 1
    pre += 1
    b = bytes(raw[pre:]) + bytes(16)
    n = len(raw) - pre
    nc = (n + CH - 1) // CH
    # truth
    T = []  # true exit per chunk
    pos = 0; starts = set()
    while pos < n:
        starts.add(pos); adv, ln, off = elem(b, pos); pos += adv
    # true entry of chunk j = first element start >= cs, or skip beyond
    true_entry = []
    pos = 0; j = 0
    srt = sorted(starts)
    import bisect
    for j in range(nc):
        cs = j * CH
        k = bisect.bisect_left(srt, cs)
        # entry = smallest true start >= cs (elements straddling chunk start skip into later)
        true_entry.append(srt[k] if k < len(srt) else n)
    # spec
    spec_exit = []; vis = []
    for j in range(nc):
        cs = j * CH; ce = min(cs + CH, n)
        p = max(cs - WU, 0); v = set()
        while p < ce:
            if p >= cs: v.add(p)
            adv, ln, off = elem(b, p); p += adv
        spec_exit.append(p); vis.append(v)
    def walk(e, ce):
        while e < ce:
            adv, ln, off = elem(b, e); e += adv
        return e
    assumed = []
    for j in range(nc):
        cs = j * CH; ce = min(cs + CH, n)
        e = 0 if j == 0 else spec_exit[j-1]
        if e >= ce: x = e
        elif j == 0 or e in vis[j]: x = spec_exit[j]
        else: x = walk(e, ce)
        assumed.append(x)
    broke = [assumed[j] != spec_exit[j] for j in range(nc)]
    entry = [None] * nc; flag = [False] * nc
    for j in range(nc):
        if j == 0: entry[j] = 0; continue
        bb = j - 1; genuine = False
        if j >= 2 and broke[bb - 1]:
            r = 0
            while r < MAX_RUN and j - 2 > r and broke[bb - 2 - r]: r += 1
            if r == MAX_RUN:
                flag[j - 2 - MAX_RUN if j - 2 > MAX_RUN else 0] = True; entry[j] = -1; continue
            genuine = (r & 1) == 0
        if not genuine: entry[j] = assumed[bb]; continue
        cs = (j - 1) * CH; ce = min(cs + CH, n)
        e = assumed[bb - 1]
        if not (e < ce and e in vis[bb]):
            flag[j - 2] = True; entry[j] = -1; continue
        entry[j] = spec_exit[bb]
    wrong = [j for j in range(nc) if entry[j] != -1 and entry[j] != true_entry[j]]
    flags = [j for j in range(nc) if flag[j]]
    return nc, wrong, flags, broke

if __name__ == "__main__":
    T0 = 1_700_000_000_000
    for V in range(0, 40):
        data = (np.arange(60000, dtype=np.int64) + T0 + V * 60000).tobytes()
        raw = pa.compress(data, codec='snappy', asbytes=True)
        for CH in (256, 128):
            nc, wrong, flags, broke = run(raw, CH)
            if wrong:
                print("V", V, "CH", CH, "n_in", len(raw), "chunks", nc, "wrong", len(wrong), wrong[:10], "flags", flags[:10], "breaks", sum(broke))

def resolve_all(raw, CH=256, WU=192, MAX_RUN=32, GAP=80, MARGIN=8, order=None):
    """entries after k_snap_entries + k_snap_regions + k_snap_resolve with regions processed one
    after another in `order` (default: ascending); returns (#regions, #wrong entries)."""
    import bisect
    pre = 0
    while raw[pre] & 0x80: pre += 1
    pre += 1
    b = bytes(raw[pre:]) + bytes(16)
    n = len(raw) - pre
    nc = (n + CH - 1) // CH
    # recompute via run() internals
    starts = []; pos = 0
    while pos < n:
        starts.append(pos); pos += elem(b, pos)[0]
    true_entry = []
    for j in range(nc):
        k = bisect.bisect_left(starts, j * CH); true_entry.append(starts[k] if k < len(starts) else n)
    spec_exit = []; vis = []
    for j in range(nc):
        cs = j * CH; ce = min(cs + CH, n); p = max(cs - WU, 0); v = set()
        while p < ce:
            if p >= cs: v.add(p)
            p += elem(b, p)[0]
        spec_exit.append(p); vis.append(v)
    def walk(e, ce):
        while e < ce: e += elem(b, e)[0]
        return e
    assumed = []
    for j in range(nc):
        cs = j * CH; ce = min(cs + CH, n); e = 0 if j == 0 else spec_exit[j-1]
        assumed.append(e if e >= ce else spec_exit[j] if (j == 0 or e in vis[j]) else walk(e, ce))
    broke = [assumed[j] != spec_exit[j] for j in range(nc)]
    entry = [0] * nc; flag = [False] * nc
    for j in range(1, nc):
        bb = j - 1; genuine = False
        if j >= 2 and broke[bb - 1]:
            r = 0
            while r < MAX_RUN and j - 2 > r and broke[bb - 2 - r]: r += 1
            if r == MAX_RUN:
                flag[j - 2 - MAX_RUN if j - 2 > MAX_RUN else 0] = True; entry[j] = 0xffffffff; continue
            genuine = (r & 1) == 0
        if not genuine: entry[j] = assumed[bb]; continue
        cs = (j - 1) * CH; ce = min(cs + CH, n); e = assumed[bb - 1]
        if not (e < ce and e in vis[bb]):
            flag[j - 2] = True; entry[j] = 0xffffffff; continue
        entry[j] = spec_exit[bb]
    regions = [c for c in range(nc) if flag[c] and not any(flag[max(0, c - GAP):c])]
    pre_entry = list(entry)
    def resolver(jf):
        base = jf - MARGIN if jf > MARGIN else 0
        yield
        e = 0 if base == 0 else entry[base]
        while base < nc:
            cnt = min(64, nc - base)
            cands = []; oks = []; olds = []
            for lane in range(cnt):
                j = base + lane; cs = j * CH; ce = min(cs + CH, n)
                cand = e if lane == 0 else spec_exit[j - 1]
                skip = cand >= ce
                ok = (not skip) and (cand in vis[j])
                cands.append(cand); oks.append(ok); olds.append(entry[j])
            f = next((l for l in range(cnt) if not oks[l]), 64)
            agree = all(min(cands[l], 0xffffffff) == olds[l] for l in range(cnt))
            yield
            for l in range(cnt):
                if l <= f: entry[base + l] = min(cands[l], 0xffffffff)
            if f >= cnt:
                if agree and base > jf and (not FIX or not any(flag[base:min(nc, base + cnt + GAP)])): break
                e = spec_exit[base + cnt - 1]; base += cnt; continue
            # r04: breaks inside the window are followed one after another without reloading it
            nxt = True
            while True:
                ef0 = cands[f]; fcs = (base + f) * CH; fce = min(fcs + CH, n)
                if ef0 >= fce:
                    jt = min(ef0 // CH, nc)
                    for q in range(base + f + 1, jt): entry[q] = ef0
                    e = ef0; base = jt if jt > base + f else base + f + 1; nxt = False; break
                ef = walk(ef0, fce)
                if f + 1 >= cnt:
                    e = ef; base += f + 1; nxt = False; break
                j1 = base + f + 1; cs1 = j1 * CH; ce1 = min(cs1 + CH, n)
                cands[f + 1] = ef
                oks[f + 1] = ef < ce1 and ef in vis[j1]
                f2 = next((l for l in range(f + 1, cnt) if not oks[l]), 64)
                for l in range(f + 1, min(f2, cnt - 1) + 1): entry[base + l] = min(cands[l], 0xffffffff)
                f = f2
                if f >= cnt: break
            if nxt:
                e = spec_exit[base + cnt - 1]; base += cnt
            yield
    if order == "interleave":
        gens = [resolver(jf) for jf in regions]
        while gens:
            nxt = []
            for g in gens:
                try:
                    next(g); nxt.append(g)
                except StopIteration:
                    pass
            gens = nxt
    else:
        if order is None: order = list(range(len(regions)))
        for ri in order:
            for _ in resolver(regions[ri]): pass
    wrong = [j for j in range(nc) if entry[j] != true_entry[j]]
    global DBG
    DBG = dict(regions=regions, flags=[c for c in range(nc) if flag[c]], entry=entry, pre_entry=pre_entry, true_entry=true_entry)
    return len(regions), wrong
