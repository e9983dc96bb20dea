"""The wave-parallel FSE table build of zd_k_fused / zd_k_tables_seqw
(zd_kernels.hip fz_build_fse) restated on the host and checked against the
serial construction (FseTable::from_distribution, fse.rs:110-202, as K1's
build_fse and the oracle walk it): placement r of the spread lands on the
r-th position j * step & mask below the -1 symbols' top positions, and a
state's nextState is count(s) plus its rank among the earlier states of s,
counted per 64 states.  Host logic only (no GPU)."""
import random


def serial_table(al, dist):
    T = 1 << al
    zero_pos, sym = T, [None] * T
    for s, c in enumerate(dist):
        if c == -1:
            zero_pos -= 1
            sym[zero_pos] = s
    pos, step, mask = 0, (T >> 1) + (T >> 3) + 3, T - 1
    for s, c in enumerate(dist):
        for _ in range(max(c, 0)):
            sym[pos] = s
            pos = (pos + step) & mask
            while pos >= zero_pos:
                pos = (pos + step) & mask
    nxt = [c if c > 0 else (1 if c == -1 else 0) for c in dist]
    out = []
    for i in range(T):
        out.append((sym[i], nxt[sym[i]]))
        nxt[sym[i]] += 1
    return out


def wave_table(al, dist):
    T = 1 << al
    mask, step = T - 1, (T >> 1) + (T >> 3) + 3
    sym, cum, nneg, placed = [None] * T, [], 0, 0
    for s, c in enumerate(dist):               # -1 symbols from the top; cumulative placements
        if c == -1:
            sym[T - 1 - nneg] = s
            nneg += 1
        cum.append(placed)
        placed += max(c, 0)
    zero_pos = T - nneg
    assert placed == zero_pos
    r = 0
    for j in range(T):                          # lanes over j, ranks by ballot prefix counts
        x = (j * step) & mask
        if x < zero_pos:
            lo, hi = 0, len(dist)               # the last symbol with cum <= r
            while hi - lo > 1:
                mid = (lo + hi) // 2
                if cum[mid] <= r:
                    lo = mid
                else:
                    hi = mid
            sym[x] = lo
            r += 1
    cnt = [c if c > 0 else (1 if c == -1 else 0) for c in dist]
    out = []
    for i0 in range(0, T, 64):                  # 64 states a round
        chunk = sym[i0:i0 + 64]
        occ = [sum(1 for l2 in range(l) if chunk[l2] == chunk[l]) for l in range(len(chunk))]
        ns = [cnt[chunk[l]] + occ[l] for l in range(len(chunk))]
        for l in range(len(chunk)):
            if occ[l] + 1 == chunk.count(chunk[l]):
                cnt[chunk[l]] = ns[l] + 1
        out += list(zip(chunk, ns))
    return out


def random_dist(r, al, nsym):
    T = 1 << al
    dist, rem = [0] * nsym, T
    while rem > 0:
        s = r.randrange(nsym)
        if r.random() < 0.1 and dist[s] == 0:
            dist[s], rem = -1, rem - 1
        elif dist[s] >= 0:
            k = min(rem, r.randint(1, max(1, rem // 3)))
            dist[s], rem = dist[s] + k, rem - k
        elif all(d < 0 for d in dist):
            dist.append(rem)
            rem = 0
    return dist


def test_wave_spread_equals_serial():
    r = random.Random(5150)
    for _ in range(400):
        al = r.randint(5, 9)
        dist = random_dist(r, al, r.choice([r.randint(1, 36), r.randint(2, 64), r.randint(65, 255)]))
        assert wave_table(al, dist) == serial_table(al, dist), (al, dist)


def test_predefined_distributions():
    ll = [4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1,
          -1, -1, -1, -1]
    of = [1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1]
    ml = [1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
          1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1]
    for al, d in ((6, ll), (5, of), (6, ml)):
        assert sum(abs(x) for x in d) == 1 << al
        assert wave_table(al, d) == serial_table(al, d)
