"""Diagnostic: the serial world with soup births, GPU twice and the oracle,
update by update (first divergence, alive maps)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_birth_soup as t  # noqa: E402
import oracle_lib as ol  # noqa: E402
from avida_amd import capi  # noqa: E402

golden = os.path.join(ROOT, "tests", "golden")
iset, env, cfg, n, g = t._serial_pair(golden, 1, 0)
bs = [ol.Backend(k, cfg, iset, env, ncells=n) for k in ("oracle", "gpu", "gpu")]
for b in bs:
    b.set_orgs(0, g, deterministic=False)
for upd in range(40):
    ss = [b.run_serial_update() for b in bs]
    vals = [(s.num_organisms, s.births, s.deaths, s.insts_executed) for s in ss]
    print(upd, vals, flush=True)
    if len(set(vals)) > 1:
        al = []
        for b in bs:
            st, _, _ = b.states(0, n, capi.MAX_GENOME)
            al.append([c for c in range(n) if st[c].mem_size > 0])
        print("alive oracle", al[0]); print("alive gpu1  ", al[1]); print("alive gpu2  ", al[2])
        break
