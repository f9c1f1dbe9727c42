"""Static spill census of the hot loops of a kernel in a gfx950 assembly listing.

Builds the CFG of the kernel's blocks, finds the natural loops, and reports for the
microstep loop (the loop that calls the noise refill) and the resolver loop (the loop
that calls the column QR solver) the number of scratch spill loads / stores, SGPR
spill lane moves and instructions in the loop body (inner loops included).  Spill
counts from -Rpass-analysis are totals over the whole kernel; this says where they sit.

    hipcc ... -S --cuda-device-only -x hip fks_kernels.hip -o k.s
    python tools/loop_spills.py k.s [kernel]
"""
from __future__ import annotations

import re
import sys
from collections import defaultdict


def kernel_lines(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end") and i > start)
    return lines[start:end]


def analyse(lines):
    blocks, cur = [], ("entry", 0)
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m:
            blocks.append((cur[0], cur[1], i))
            cur = (m.group(1), i)
    blocks.append((cur[0], cur[1], len(lines)))
    idx = {b[0]: k for k, b in enumerate(blocks)}
    succ = defaultdict(set)
    for k, (lab, s, e) in enumerate(blocks):
        uncond = False
        for l in lines[s:e]:
            m = re.search(r"\ts_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", l)
            if m:
                succ[k].add(idx[m.group(2)])
                uncond = uncond or m.group(1) == "branch"
            if re.search(r"\ts_endpgm", l):
                uncond = True
        if not uncond and k + 1 < len(blocks):
            succ[k].add(k + 1)
    n = len(blocks)
    preds = defaultdict(set)
    for u in range(n):
        for w in succ[u]:
            preds[w].add(u)
    # iterative dominators (reverse post-order)
    order, seen = [], set()
    stack = [(0, iter(sorted(succ[0])))]
    seen.add(0)
    while stack:
        v, it = stack[-1]
        nxt = next(it, None)
        if nxt is None:
            order.append(v)
            stack.pop()
        elif nxt not in seen:
            seen.add(nxt)
            stack.append((nxt, iter(sorted(succ[nxt]))))
    rpo = order[::-1]
    pos = {v: i for i, v in enumerate(rpo)}
    dom = {rpo[0]: rpo[0]}

    def intersect(a, b):
        while a != b:
            while pos[a] > pos[b]:
                a = dom[a]
            while pos[b] > pos[a]:
                b = dom[b]
        return a

    changed = True
    while changed:
        changed = False
        for v in rpo[1:]:
            ps = [p for p in preds[v] if p in dom]
            if not ps:
                continue
            d = ps[0]
            for p in ps[1:]:
                d = intersect(p, d)
            if dom.get(v) != d:
                dom[v] = d
                changed = True

    def dominates(a, b):
        while True:
            if a == b:
                return True
            if b == dom.get(b, b):
                return False
            b = dom[b]

    loops = defaultdict(set)
    for u in range(n):
        for h in succ[u]:
            if u in dom and h in dom and dominates(h, u):
                body, st = {h, u}, [u]
                while st:
                    x = st.pop()
                    for p in preds[x]:
                        if p not in body:
                            body.add(p)
                            st.append(p)
                loops[h] |= body
    return blocks, loops


def census(lines, blocks, body):
    c = defaultdict(int)
    for k in body:
        _, s, e = blocks[k]
        for l in lines[s:e]:
            t = l.strip()
            if not t or t.startswith(";") or t.endswith(":") or t.startswith("."):
                continue
            c["insts"] += 1
            for key in ("scratch_load", "scratch_store", "v_readlane", "v_writelane", "s_load", "global_load", "ds_read",
                        "s_waitcnt", "s_swappc"):
                if t.startswith(key):
                    c[key] += 1
            if t.startswith("v_") and not t.startswith(("v_readlane", "v_writelane")):
                c["valu"] += 1
    return dict(c)


def main():
    path = sys.argv[1]
    name = sys.argv[2] if len(sys.argv) > 2 else "fks_simulate_linked"
    lines = kernel_lines(path, name)
    blocks, loops = analyse(lines)

    def calls(body, pat):
        return any(pat in l for k in body for l in lines[blocks[k][1]:blocks[k][2]] if "s_swappc" in l or "s_getpc" in l or
                   "rel32@lo" in l)

    def loop_with(pat):
        cands = [(len(b), h, b) for h, b in loops.items() if calls(b, pat)]
        return min(cands)[1:] if cands else (None, set())

    for label, pat in (("microstep loop", "refill_noise_lanes"), ("resolver loop", "qr_solve_cols")):
        h, body = loop_with(pat)
        if h is None:
            print(label, "not found (callee inlined?)")
            continue
        print(f"{label}: header {blocks[h][0]}, {len(body)} blocks", census(lines, blocks, body))
    # the largest loops whatever they call: with everything inlined the hot loops are
    # the few nests of several hundred blocks
    print("largest loops:")
    for size, h in sorted(((len(b), h) for h, b in loops.items()), reverse=True)[:6]:
        print(f"  header {blocks[h][0]}, {size} blocks", census(lines, blocks, loops[h]))


if __name__ == "__main__":
    main()
