import sys, numpy as np
exec(open(__file__.replace("nd_probe", "order_probe").replace("rounds_probe", "order_probe")).read().split("def elim_order_min_degree")[0])
def simulate(adj, dcap, rmin, mmd, rmax=64):
    A = [set(s) for s in adj]; alive = set(range(len(A))); rounds = []
    while alive and len(rounds) < rmax:
        if all(len(A[v]) == len(alive) - 1 for v in alive): break
        dmin = min(len(A[v]) for v in alive)
        dlim = min(dcap, max(2 * dmin, dmin + 1)) if mmd else dcap
        cand = sorted([v for v in alive if len(A[v]) <= dlim], key=lambda v: len(A[v]))
        blocked = set(); chosen = []
        for v in cand:
            if v in blocked: continue
            chosen.append(v); blocked.add(v); blocked |= A[v]
        if len(chosen) < rmin and len(chosen) != len(alive): break
        fr = [len(A[v]) for v in chosen]
        rounds.append((len(chosen), max(fr) if fr else 0))
        for v in chosen:
            nb = A[v]
            for a in nb:
                A[a] |= nb; A[a].discard(a); A[a].discard(v)
            A[v] = set(); alive.discard(v)
    return rounds, len(alive)
for dcap, rmin, mmd in [(16,2,0),(24,2,0),(32,2,0),(64,2,0),(16,2,1),(32,2,1),(64,2,1),(64,4,1),(64,6,1),(64,8,1),(100,6,0)]:
    r, core = simulate(adj, dcap, rmin, mmd)
    ncol = (7*core + 63)//64
    cost = len(r) * 10.4 + ncol * 16.4
    print(f"dcap {dcap:3d} rmin {rmin} mmd {mmd}: rounds {len(r):2d} core {core:3d} ({ncol} tile cols) est {cost:.0f} us  rounds={r}")
