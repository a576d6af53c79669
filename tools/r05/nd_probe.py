import sys, numpy as np
exec(open(__file__.replace("nd_probe", "order_probe").replace("rounds_probe", "order_probe")).read().split("order = elim_order_min_degree")[0])
import scipy.sparse as sp, scipy.sparse.linalg as sla

def sep_split(nodes, adj):
    nodes = list(nodes)
    if len(nodes) <= 12: return None
    idx = {v: i for i, v in enumerate(nodes)}
    m = len(nodes)
    L = np.zeros((m, m))
    for v in nodes:
        for u in adj[v]:
            if u in idx:
                L[idx[v], idx[u]] = -1
    L += np.diag(-L.sum(1))
    w, V = np.linalg.eigh(L)
    f = V[:, 1]
    best = None
    for q in np.linspace(0.3, 0.7, 21):
        thr = np.quantile(f, q)
        A = set(nodes[i] for i in range(m) if f[i] < thr); B = set(nodes) - A
        # vertex separator: greedy min vertex cover of cut edges (bipartite: take from side with fewer endpoints)
        cut = [(a, b) for a in A for b in adj[a] if b in B]
        S = set()
        # greedy vertex cover by max degree in cut graph
        cg = {}
        for a, b in cut:
            cg.setdefault(a, set()).add(b); cg.setdefault(b, set()).add(a)
        while any(cg.values()):
            v = max(cg, key=lambda x: len(cg[x]))
            S.add(v)
            for u in cg[v]: cg[u].discard(v)
            cg[v] = set()
        A2, B2 = A - S, B - S
        score = len(S) + max(len(A2), len(B2)) * 0.0
        cost = len(S) + 0.5 * abs(len(A2) - len(B2)) * 0
        key = (len(S) + max(len(A2), len(B2)))  # rough critical path proxy
        if best is None or key < best[0]:
            best = (key, A2, B2, S)
    return best[1], best[2], best[3]

def nd(nodes, adj, depth=0):
    r = sep_split(nodes, adj)
    if r is None:
        return [list(nodes)], 0
    A, B, S = r
    if not A or not B or len(A) + len(B) + len(S) != len(nodes) or len(S) >= len(nodes) - 2:
        return [list(nodes)], 0
    oa, _ = nd(A, adj, depth + 1); ob, _ = nd(B, adj, depth + 1)
    return oa + ob + [list(S)], 0

groups, _ = nd(set(range(n)), adj)
order = [v for g in groups for v in g]
parent, cc, h = etree_stats(adj, order)
print("ND: etree height", max(h.values()), "fill", sum(cc.values()))
top = groups[-1]
print("top separator size", len(top))
# critical path with min-degree inside leaves
