"""Premultiplier split for the squaring columns (edv_math.h kSqSplit).

Term f_i f_j (i <= j) of f^2 (or 2 f^2) carries the constant
M = (2 if i < j) * (2 if i, j both odd) * (19 if i + j >= 10) * (2 if DOUBLE).
The kernel multiplies (x * f_i) * (y * f_j) with x * y = M, where x * f_i must
stay inside int32 under the multiply's input bound (|f| <= 1.65 * 2^26 even,
1.65 * 2^25 odd limbs), i.e. x <= 19 on even limbs and x <= 38 on odd limbs.
Every distinct (limb, multiplier != 1) pair costs one instruction per square,
so this picks the split minimising their number (a small 0/1 ILP, scipy milp).
Prints the C++ table.  Result: 13 premultiplied operands for f^2 (17 with the
earlier hand rule), 21 for 2 f^2 (27).
"""
import numpy as np
from scipy.optimize import Bounds, LinearConstraint, milp


def solve(double):
    terms = []
    for i in range(10):
        for j in range(i, 10):
            m = (2 if i < j else 1) * (2 if (i & 1) and (j & 1) else 1) * (19 if i + j >= 10 else 1)
            terms.append((i, j, m * (2 if double else 1)))
    cap = lambda l: 38 if l & 1 else 19
    splits = [[(x, m // x) for x in range(1, m + 1) if m % x == 0 and x <= cap(i) and m // x <= cap(j)]
              for (i, j, m) in terms]
    pairs = sorted({p for t, (i, j, m) in enumerate(terms) for (x, y) in splits[t]
                    for p in ((i, x), (j, y)) if p[1] != 1})
    pid = {p: k for k, p in enumerate(pairs)}
    yv = [(t, s) for t in range(len(terms)) for s in range(len(splits[t]))]
    nz, n = len(pairs), len(pairs) + len(yv)
    rows, lb, ub = [], [], []
    for t in range(len(terms)):
        row = np.zeros(n)
        for k, (tt, s) in enumerate(yv):
            if tt == t:
                row[nz + k] = 1
        rows.append(row); lb.append(1); ub.append(1)
    for k, (t, s) in enumerate(yv):
        i, j, _ = terms[t]
        x, y = splits[t][s]
        for p in ((i, x), (j, y)):
            if p[1] != 1:
                row = np.zeros(n); row[nz + k] = 1; row[pid[p]] = -1
                rows.append(row); lb.append(-np.inf); ub.append(0)
    res = milp(np.concatenate([np.ones(nz), np.zeros(len(yv))]),
               constraints=LinearConstraint(np.array(rows), lb, ub),
               integrality=np.ones(n), bounds=Bounds(0, 1))
    table = [[(0, 0)] * 10 for _ in range(10)]
    for k, (t, s) in enumerate(yv):
        if res.x[nz + k] > 0.5:
            i, j, _ = terms[t]
            table[i][j] = splits[t][s]
    return int(round(res.fun)), table


if __name__ == "__main__":
    for d in (False, True):
        cost, table = solve(d)
        print("// %s: %d premultiplied operands" % ("2 f^2" if d else "f^2", cost))
        for i in range(10):
            print("    {" + ", ".join("{%d, %d}" % table[i][j] for j in range(10)) + "},")
