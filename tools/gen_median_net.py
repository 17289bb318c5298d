#!/usr/bin/env python3
"""Generate straight-line k×k median selection networks for the gfx950 median kernel.

Design (Adams 2021 "separable sorting networks" idea, re-derived here):
  * A thread owns a TW×TH tile of outputs; its inputs are the (TW+k-1)×(TH+k-1) window union.
  * Vertical stage: for every input column, the k-row windows of the TH output rows share a
    core of rows; a binary tree over the output rows sorts the core once and merges the extra
    rows in as the tree descends (Batcher odd-even merges for arbitrary lengths).
  * Horizontal stage: the same tree over output columns merges whole sorted columns.
  * Leaves select rank (k²-1)/2 from (parent list, extra list) with the exact min/max formula
    kth(A,B) = min_i max(A[i-1], B[k-i-1]).
  * Hash-consing (CSE) shares every identical min/max across the tile; dead-code elimination
    keeps only what feeds the TW·TH medians.
Each op is one v_pk_min_u16 / v_pk_max_u16 on a packed pair of pixels, so a thread computes
2·TW·TH medians (its tile and the tile half a workgroup-tile to the right).

Usage: python tools/gen_median_net.py --emit include/nm03/median_net.inc
       python tools/gen_median_net.py --explore
"""
import argparse
import itertools
import sys

INF, NINF = "INF", "NINF"


class Net:
    def __init__(self):
        self.nodes = []  # (op, a, b) ; op in {'in','min','max'}
        self.index = {}

    def inp(self, r, c):
        key = ("in", r, c)
        if key not in self.index:
            self.index[key] = len(self.nodes)
            self.nodes.append(key)
        return self.index[key]

    def op(self, op, a, b):
        if a == b:
            return a
        if a == INF or b == INF:
            if op == "min":
                return b if a == INF else a
            return INF
        if a == NINF or b == NINF:
            if op == "max":
                return b if a == NINF else a
            return NINF
        if a > b:
            a, b = b, a
        # absorption: max(a, min(a,b)) = a, min(a, max(a,b)) = a
        for x, y in ((a, b), (b, a)):
            n = self.nodes[y]
            if n[0] in ("min", "max") and x in (n[1], n[2]):
                if op == "max" and n[0] == "min":
                    return x
                if op == "min" and n[0] == "max":
                    return x
                if op == n[0]:
                    return y  # min(a, min(a,b)) = min(a,b)
        key = (op, a, b)
        if key not in self.index:
            self.index[key] = len(self.nodes)
            self.nodes.append(key)
        return self.index[key]

    def cx(self, a, b):
        return self.op("min", a, b), self.op("max", a, b)


def merge(net, A, B):
    """Batcher odd-even merge of two sorted lists of arbitrary length."""
    if not A:
        return list(B)
    if not B:
        return list(A)
    if len(A) == 1 and len(B) == 1:
        return list(net.cx(A[0], B[0]))
    v = merge(net, A[0::2], B[0::2])
    w = merge(net, A[1::2], B[1::2])
    seq = []
    for i in range(max(len(v), len(w))):
        if i < len(v):
            seq.append(v[i])
        if i < len(w):
            seq.append(w[i])
    # compare-exchange pairs (w_i, v_{i+1}) at positions (2i+1, 2i+2)
    for i in range(len(w)):
        p = 2 * i + 1
        if p + 1 < len(seq):
            seq[p], seq[p + 1] = net.cx(seq[p], seq[p + 1])
    return seq


def sort(net, L):
    if len(L) <= 1:
        return list(L)
    h = len(L) // 2
    return merge(net, sort(net, L[:h]), sort(net, L[h:]))


def merge_many(net, lists):
    lists = [l for l in lists if l]
    while len(lists) > 1:
        nxt = []
        # merge smallest first for balance
        lists.sort(key=len)
        for i in range(0, len(lists) - 1, 2):
            nxt.append(merge(net, lists[i], lists[i + 1]))
        if len(lists) % 2:
            nxt.append(lists[-1])
        lists = nxt
    return lists[0] if lists else []


def kth(net, A, B, t):
    """t-th smallest (0-based) of A ∪ B, both sorted: min over splits of max(A[i-1], B[j-1])."""
    k = t + 1
    m, n = len(A), len(B)
    cands = []
    for i in range(max(0, k - n), min(m, k) + 1):
        j = k - i
        a = A[i - 1] if i > 0 else NINF
        b = B[j - 1] if j > 0 else NINF
        cands.append(net.op("max", a, b))
    r = cands[0]
    for c in cands[1:]:
        r = net.op("min", r, c)
    return r


def tree(net, lo, hi, k, items_for, parent_sorted, parent_range, leaf_fn):
    """Recursive shared-core tree over output indices [lo,hi).

    items_for(range_start, range_end) returns the unsorted 'new' lists for indices covered by the
    core of [lo,hi) but not by the parent's core. Core of [a,b) = [b-1, a+k-1].
    """
    core = (hi - 1, lo + k - 1)
    if parent_range is None:
        new_idx = list(range(core[0], core[1] + 1))
    else:
        pc = parent_range
        new_idx = [x for x in range(core[0], core[1] + 1) if not (pc[0] <= x <= pc[1])]
    new_sorted = merge_many(net, [items_for(x) for x in new_idx])
    if hi - lo == 1:
        return leaf_fn(lo, parent_sorted if parent_sorted is not None else [], new_sorted)
    cur = merge(net, parent_sorted, new_sorted) if parent_sorted is not None else new_sorted
    mid = (lo + hi) // 2
    out = {}
    out.update(tree(net, lo, mid, k, items_for, cur, core, leaf_fn))
    out.update(tree(net, mid, hi, k, items_for, cur, core, leaf_fn))
    return out


def build(k, TW, TH):
    net = Net()
    t = (k * k - 1) // 2
    # Vertical stage: sorted column windows col_sorted[(row_out, c)]
    col_sorted = {}
    for c in range(TW + k - 1):

        def items_col(r, c=c):
            return [net.inp(r, c)]

        def leaf_col(i, parent, new, c=c):
            return {(i, c): merge(net, parent, new)}

        col_sorted.update(tree(net, 0, TH, k, items_col, None, None, leaf_col))
    outs = {}
    for i in range(TH):

        def items_row(c, i=i):
            return col_sorted[(i, c)]

        def leaf_row(j, parent, new, i=i):
            return {(i, j): kth(net, parent, new, t)}

        outs.update(tree(net, 0, TW, k, items_row, None, None, leaf_row))
    return net, outs


def live_ops(net, outs):
    need = set()
    stack = [v for v in outs.values() if isinstance(v, int)]
    while stack:
        x = stack.pop()
        if x in need:
            continue
        need.add(x)
        n = net.nodes[x]
        if n[0] != "in":
            for y in (n[1], n[2]):
                if isinstance(y, int):
                    stack.append(y)
    ops = sorted(x for x in need if net.nodes[x][0] != "in")
    ins = sorted(x for x in need if net.nodes[x][0] == "in")
    return ops, ins


def demand_order(net, outs):
    """Post-order DFS from the outputs in output order: every value (input load included) is
    produced just before its first consumer, so the live set stays near the sorted columns the
    remaining outputs still need — instead of creation order, which loads every input and sorts
    every column before the first horizontal merge (peak ≈ all inputs live; the k=7 kernel needed
    139 VGPRs = 3 waves/SIMD)."""
    order, seen = [], set()
    for _, root in sorted(outs.items()):
        if not isinstance(root, int) or root in seen:
            continue
        stack = [(root, False)]
        while stack:
            x, done = stack.pop()
            if done:
                order.append(x)
                continue
            if x in seen:
                continue
            seen.add(x)
            stack.append((x, True))
            n = net.nodes[x]
            if n[0] != "in":
                for y in (n[2], n[1]):
                    if isinstance(y, int) and y not in seen:
                        stack.append((y, False))
    return order


def emit(k, TW, TH, f):
    net, outs = build(k, TW, TH)
    ops, ins = live_ops(net, outs)
    name = f"median_net_k{k}_w{TW}_h{TH}"
    f.write(f"// {name}: {len(ops)} packed min/max ops for {TW*TH} outputs "
            f"({len(ops)/(TW*TH):.1f} ops/output, 2 pixels per op)\n")
    f.write(f"#define NM03_{name.upper()}_OPS {len(ops)}\n")
    f.write("template <class V, class LD>\n")
    f.write(f"NM03_HD void {name}(const LD& ld, V* out) {{\n")
    var = {}
    for x in demand_order(net, outs):
        n = net.nodes[x]
        if n[0] == "in":
            var[x] = f"i{n[1]}_{n[2]}"
            f.write(f"  const V {var[x]} = ld({n[1]}, {n[2]});\n")
            continue
        op, a, b = n
        var[x] = f"t{x}"
        fn = "vmin" if op == "min" else "vmax"
        f.write(f"  const V {var[x]} = {fn}({var[a]}, {var[b]});\n")
    for (i, j), v in sorted(outs.items()):
        f.write(f"  out[{i * TW + j}] = {var[v]};\n")
    f.write("}\n\n")
    return len(ops)


def verify(k, TW, TH, trials=300):
    import random
    net, outs = build(k, TW, TH)
    rnd = random.Random(1)
    for trial in range(trials):
        H, W = TH + k - 1, TW + k - 1
        hi = rnd.choice([3, 50, 65535])
        img = [[rnd.randint(0, hi) for _ in range(W)] for _ in range(H)]
        val = {}
        for x, n in enumerate(net.nodes):
            if n[0] == "in":
                val[x] = img[n[1]][n[2]]
            else:
                a = val[n[1]] if isinstance(n[1], int) else (10**9 if n[1] == INF else -1)
                b = val[n[2]] if isinstance(n[2], int) else (10**9 if n[2] == INF else -1)
                val[x] = min(a, b) if n[0] == "min" else max(a, b)
        for (i, j), v in outs.items():
            win = sorted(img[i + r][j + c] for r in range(k) for c in range(k))
            if val[v] != win[(k * k - 1) // 2]:
                raise SystemExit(f"network k={k} {TW}x{TH} wrong at trial {trial} out {(i, j)}")
    return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--explore", action="store_true")
    ap.add_argument("--emit")
    args = ap.parse_args()
    if args.explore:
        for k in (3, 5, 7, 9):
            for TW, TH in itertools.product((1, 2, 4, 8), (1, 2, 4, 8)):
                net, outs = build(k, TW, TH)
                ops, ins = live_ops(net, outs)
                print(f"k={k} TW={TW} TH={TH}: ops={len(ops):5d} ins={len(ins):4d} "
                      f"ops/px={len(ops)/(TW*TH):6.1f}", flush=True)
        return
    if args.emit:
        configs = {3: (8, 1), 5: (8, 1), 7: (8, 1), 9: (8, 1)}
        with open(args.emit, "w") as f:
            f.write("// GENERATED by tools/gen_median_net.py — do not edit.\n")
            f.write("// Straight-line median selection networks (CSE + DCE'd Batcher merge trees).\n")
            f.write("#pragma once\n\n")
            for k, (TW, TH) in configs.items():
                verify(k, TW, TH)
                n = emit(k, TW, TH, f)
                print(f"k={k} {TW}x{TH}: {n} ops ({n/(TW*TH):.1f}/px)")


if __name__ == "__main__":
    main()
