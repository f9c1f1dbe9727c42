"""Spill sites of the hot loops by source line: scratch stores / loads of the microstep loop
(without the resolver loop inside it), the resolver loop and the controller-step loop (without
the microstep loop), each with the .loc line it follows.  Needs a line-table build:

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -gline-tables-only -Iinclude \
          -Ifast_kinematic_simulator_amd/csrc --cuda-device-only -S -x hip \
          fast_kinematic_simulator_amd/csrc/fks_kernels.hip -o k.s
    python tools/spill_sites.py k.s
"""
import os
import re
import sys
from collections import Counter

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import loop_spills as L  # noqa: E402

path = sys.argv[1]
lines = L.kernel_lines(path, sys.argv[2] if len(sys.argv) > 2 else 'fks_simulate_shaped')
blocks, loops = L.analyse(lines)
def calls(body, pat):
    return any(pat in l for k in body for l in lines[blocks[k][1]:blocks[k][2]] if "rel32@lo" in l)
def loop_with(pat):
    c = [(len(b), h, b) for h, b in loops.items() if calls(b, pat)]
    return min(c)[1:]
hm, micro = loop_with('refill_noise_lanes')
hr, resol = loop_with('qr_solve_cols')
# the loop nest that contains the step loop: smallest loop strictly containing micro
step = min((len(b), h, b) for h, b in loops.items() if micro < b)[2]
def sites(body, exclude):
    out = Counter()
    for k in sorted(body - exclude):
        loc = None
        _, s, e = blocks[k]
        # find the last .loc before this block start
        for i in range(s, -1, -1):
            m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', lines[i])
            if m: loc = (int(m.group(1)), int(m.group(2))); break
        for l in lines[s:e]:
            m = re.match(r'\s*\.loc\s+(\d+)\s+(\d+)', l)
            if m: loc = (int(m.group(1)), int(m.group(2)))
            t = l.strip()
            if t.startswith('scratch_store') or t.startswith('scratch_load'):
                out[(loc, t.split()[0])] += 1
    return out
for name, body, ex in (('microstep (excl resolver)', micro, resol), ('resolver', resol, set()), ('step (excl micro)', step, micro)):
    c = sites(body, ex)
    print('==', name, sum(v for (l, k), v in c.items() if 'store' in k), 'stores', sum(v for (l, k), v in c.items() if 'load' in k), 'loads')
    for (loc, kind), v in sorted(c.items(), key=lambda x: (x[0][0] or (0, 0))):
        print('  ', loc, kind, v)
