"""Diagnostic: the configs[3] 4096x4096 world, GPU vs oracle after U updates;
prints, for each differing cell, the seeded genome length, the memory sizes and
the first differing memory sites (op / flag on both sides).
usage (GPU box): python tools/diag_config3.py [side] [updates]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as ol          # noqa: E402
import parity_util as pu         # noqa: E402
from test_parity_full import _bench_seed, _seed   # noqa: E402


def main():
    side = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    U = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    golden = os.path.join(ROOT, "tests", "golden")
    cfg, iset, env, idx, gen, glen, gmer = _bench_seed(golden, side, side)
    n = side * side
    gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
    orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
    for b in (gpu, orc):
        _seed(b, 0, idx, gen, glen, gmer)
    for u in range(U):
        sg, so = gpu.run_update(), orc.run_update()
        print("update", u, "gpu insts", sg.insts_executed, "oracle insts", so.insts_executed, flush=True)
        nbad, cells = pu.compare_digests(gpu.digests(), orc.digests(), 0, limit=40)
        print("differing cells", nbad, cells, flush=True)
        for c in cells[:12]:
            a, oa, fa = gpu.states(c, 1)
            b, ob, fb = orc.states(c, 1)
            ma, mb = a[0].mem_size, b[0].mem_size
            diff = [k for k in range(min(ma, mb)) if oa[k] != ob[k] or fa[k] != fb[k]]
            fields = [k for k in pu.STATE_FIELDS if pu.state_tuple(a[0])[k] != pu.state_tuple(b[0])[k]]
            print(f"cell {c} row {c // side} col {c % side} seeded_len {glen[idx[c]]} mem gpu {ma} orc {mb}"
                  f" fields {fields} ndiff {len(diff)} first {diff[:8]}")
            print("   gpu", [(k, oa[k], fa[k]) for k in diff[:8]])
            print("   orc", [(k, ob[k], fb[k]) for k in diff[:8]])
            print("   heads", list(a[0].head), list(b[0].head), "rng", a[0].rng_counter, b[0].rng_counter,
                  "copied", a[0].copied_size, b[0].copied_size, "cycles", a[0].cpu_cycles_used)
        if nbad:
            break


if __name__ == "__main__":
    main()
