# event simulation of the balanced unit distribution (chroma_kernel, fused step)
import heapq, random
def sim(n_units, G=256, W=16, CH=16, R=16, P=8, seed=0, slow=None):
    rnd = random.Random(seed)
    pool_lo = [n_units * x // P for x in range(P + 1)]
    pools = [0] * P
    done = [0] * n_units
    t = 0.0
    # per WG state
    class WG: pass
    wgs = []
    ev = []  # (time, seq, wg, wave, action)
    seq = [0]
    def push(tm, g, w, act):
        seq[0] += 1; heapq.heappush(ev, (tm, seq[0], g, w, act))
    for b in range(G):
        g = WG(); g.home = b % P; g.first = g.home; g.empty = set(); g.k = 0; g.ring = {}  # slot -> (tag, base, n)
        g.speed = (slow or {}).get(b % P, 1.0)
        wgs.append(g)
        # initial two chunks from home
        ordv = pools[g.home]; pools[g.home] += 2
        for c in range(2):
            bb = pool_lo[g.home] + (ordv + c) * CH
            if bb < pool_lo[g.home + 1]:
                n = min(CH, pool_lo[g.home + 1] - bb)
            else:
                bb, n = grab(g, pools, pool_lo, CH, P)
            g.ring[c % R] = (c + 1, bb, n)
        for w in range(W):
            push(rnd.random() * 1e-3, b, w, 'pull')
    def grab_now(g):
        return grab(g, pools, pool_lo, CH, P)
    ends = [0.0] * G
    while ev:
        tm, _, b, w, act = heapq.heappop(ev)
        g = wgs[b]
        if act == 'pull':
            k = g.k; g.k += 1
            c, o = divmod(k, CH)
            if o == 0:
                bb, n = grab_now(g)
                # the ring write lands after a latency
                push(tm + rnd.uniform(0.5, 3.0), b, w, ('ring', c + 2, bb, n))
            push(tm, b, w, ('read', c, o, 0))
        elif act[0] == 'ring':
            _, c, bb, n = act
            old = g.ring.get(c % R)
            assert old is None or old[0] < c + 1, "ring overwrite before read?"
            g.ring[c % R] = (c + 1, bb, n)
        elif act[0] == 'read':
            _, c, o, polls = act
            e = g.ring.get(c % R)
            if e is None or e[0] != c + 1:
                assert e is None or e[0] < c + 1, ("overwritten", c, e)
                assert polls < 10000, "stuck"
                push(tm + 0.05, b, w, ('read', c, o, polls + 1)); continue
            _, bb, n = e
            if n == 0:
                ends[b] = max(ends[b], tm); continue
            if o >= n:
                push(tm, b, w, 'pull'); continue
            u = bb + o
            done[u] += 1
            push(tm + rnd.uniform(30, 36) / g.speed, b, w, 'pull')
    assert all(d == 1 for d in done), (sum(1 for d in done if d != 1), n_units)
    return max(ends), sorted(ends)
def grab(g, pools, pool_lo, CH, P):
    for i in range(P):
        x = (g.first + i) % P
        if x in g.empty: continue
        ordv = pools[x]; pools[x] += 1
        bb = pool_lo[x] + ordv * CH
        if bb < pool_lo[x + 1]:
            g.first = x
            return bb, min(CH, pool_lo[x + 1] - bb)
        g.empty.add(x)
    return 0, 0
for n in (61440, 61440 + 7, 15, 100, 1100 * 15, 3 * 15):
    for G in (256, 3, 1):
        if G > max(1, n // 15): continue
        e, ends = sim(n, G=G, seed=n + G)
        print(n, G, round(e, 1))
# XCD 0 9% slower, XCD 1 8% faster: static would end at ~ 240/16*33/0.91
e, ends = sim(61440, slow={0: 0.91, 1: 1.08, 2: 1.06}, seed=1)
print("imbalanced XCDs: end", round(e, 1), "static share would need", round(240 / 16 * 33 / 0.91, 1))
