import sys, numpy as np
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "mast3r-slam_amd"))
from m3s import synth
N, E = 256, 1024
und = synth.make_edges(N, E, 4)
# free poses 1..255 (pose 0 pinned -> removed)
n = N - 1
adj = [set() for _ in range(n)]
for a, b in und:
    if a == 0 or b == 0: continue
    adj[a-1].add(b-1); adj[b-1].add(a-1)
deg = [len(s) for s in adj]
print("free poses", n, "edges among free", sum(deg)//2, "deg min/mean/max", min(deg), np.mean(deg), max(deg))

def elim_order_min_degree(adj):
    A = [set(s) for s in adj]; alive = set(range(len(A))); order = []
    while alive:
        v = min(alive, key=lambda x: (len(A[x]), x))
        nb = A[v]
        for a in nb:
            A[a] |= nb; A[a].discard(a); A[a].discard(v)
        alive.discard(v); order.append(v); A[v] = set()
    return order

def etree_stats(adj, order):
    pos = {v: i for i, v in enumerate(order)}
    A = [set(s) for s in adj]
    parent = {}; colcount = {}
    for v in order:
        nb = A[v]
        colcount[v] = len(nb)
        for a in nb:
            A[a] |= nb; A[a].discard(a); A[a].discard(v)
        parent[v] = min(nb, key=lambda x: pos[x]) if nb else None
        A[v] = set()
    # critical path with cost per node = 1 (pivot) -- the chain length in pivots -- and
    # weighted: cost = pivot + (front size)/64 stand-in
    depth = {}
    for v in order:
        pass
    # height of etree
    h = {}
    for v in order:
        h[v] = 1 + max([h[c] for c in order if parent.get(c) == v] or [0])
    return parent, colcount, h

order = elim_order_min_degree(adj)
parent, cc, h = etree_stats(adj, order)
root_h = max(h.values())
print("min-degree: etree height (pivots on the longest path)", root_h, " fill nnz", sum(cc.values()))
# the final clique: trailing nodes whose colcount == remaining - 1
k = 0
for i, v in enumerate(reversed(order)):
    if cc[v] == i: k = i + 1
    else: break
print("min-degree final dense clique size", k)
