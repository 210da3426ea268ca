"""Window counts of the half-size scalars, simulated in Python integers.

For random h < L: the prep kernel's rule (Euclid on (8L, h) down to the first
remainder below 2^128, the shorter odd-b neighbour) and,
for comparison, the best odd-b vector among small combinations of a
Lagrange-reduced basis.  Prints, per rule, how many lanes need each number of
signed windows of WIDTH bits (default 4, the kernel's kAWin; 5 for the earlier
layout) and how many 64-lane waves do (the main kernel walks each wave's
maximum).  Used to check that no choice of (a, b) shortens the walk:
  python tools/lattice_windows.py [lanes] [width]
"""
import collections
import random
import sys

L = 2**252 + 27742317777372353535851937790883648493
M = 8 * L


WIDTH = 4


def windows(v):
    """Windows the recode_signed<WIDTH, ...> digits of v need (1 + top nonzero digit)."""
    nd = (255 + WIDTH - 1) // WIDTH
    carry, top = 0, 0
    for k in range(nd):
        e = ((v >> (WIDTH * k)) & ((1 << WIDTH) - 1)) + carry
        carry = 0 if k == nd - 1 else (e + (1 << (WIDTH - 1))) >> WIDTH
        e -= carry << WIDTH
        if e:
            top = k + 1
    return top


def kernel_rule(h):
    """half_scalars() in edv_verify_core.h: -> (a, b), a = b h mod 8L, b odd."""
    r0, r1, t0, t1 = M, h, 0, 1
    while r1 >= 2**128:
        q = r0 // r1
        r0, r1, t0, t1 = r1, r0 - q * r1, t1, t0 - q * t1
    blen = lambda x: max(x[0].bit_length(), abs(x[1]).bit_length())
    cur, prev = (r1, t1), (r0, t0)
    if t1 & 1 and (not t0 & 1 or blen(cur) <= blen(prev)):
        return cur
    best = prev
    if not t1 & 1 and r1 >= 2**64:
        q = r0 // r1
        nxt = (r0 - q * r1, t0 - q * t1)
        if blen(nxt) < blen(prev):
            best = nxt
    return best


def best_rule(h, span=6):
    """Shortest odd-b vector (in windows) among i v1 + j v2, |i|, |j| <= span."""
    n = lambda x: x[0] * x[0] + x[1] * x[1]
    u, v = (M, 0), (h, 1)
    if n(u) < n(v):
        u, v = v, u
    while True:
        q = (2 * (u[0] * v[0] + u[1] * v[1]) + n(v)) // (2 * n(v))
        u = (u[0] - q * v[0], u[1] - q * v[1])
        if n(u) >= n(v):
            break
        u, v = v, u
    best = None
    for i in range(-span, span + 1):
        for j in range(-span, span + 1):
            a, b = i * v[0] + j * u[0], i * v[1] + j * u[1]
            if b % 2 == 0:
                continue
            if a < 0:
                a, b = -a, -b
            w = max(windows(a), windows(abs(b)))
            if best is None or w < best[0]:
                best = (w, a, b)
    return best[1], best[2]


def main():
    global WIDTH
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64 * 1024
    WIDTH = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rng = random.Random(1)
    hs = [rng.randrange(L) for _ in range(n)]
    for rule in (kernel_rule, best_rule):
        wl = []
        for h in hs:
            a, b = rule(h)
            assert (a - b * h) % M == 0 and b % 2
            wl.append(max(windows(a), windows(abs(b))))
        lanes = sorted(collections.Counter(wl).items())
        waves = sorted(collections.Counter(max(wl[k:k + 64]) for k in range(0, n, 64)).items())
        print("%-12s lanes %s  waves %s" % (rule.__name__, lanes, waves))


if __name__ == "__main__":
    main()
