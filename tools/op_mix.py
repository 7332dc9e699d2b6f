"""Dynamic instruction mix of the bench population (diagnostic).

Steps a random sample of the configs[2] seed organisms (detail-50000.pop,
classic instset, logic-9 world) one instruction at a time on the CPU oracle
and counts the op at each organism's IP -- the mix that decides which ops the
interpreter runs in its branch-free block and which it parks for the slow
phase:

  python tools/op_mix.py [organisms=256] [steps=1500]
"""
import collections
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)
from avida_amd import capi  # noqa: E402
import oracle_lib as ol  # noqa: E402
import parity_util as pu  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
    golden = os.path.join(ROOT, "tests", "golden")
    iset, env, cfg = pu.load_env(golden, instset="instset-classic.cfg", seed=5)
    random.seed(1)
    sample = random.sample(pu.pop_genomes(golden, iset), n)
    o = ol.Backend("oracle", cfg, iset, env, ncells=n)
    o.set_orgs(0, sample, deterministic=False)
    cnt = collections.Counter()
    for _ in range(steps):
        st, ops, _fl = o.states(0, n)
        for i in range(n):
            if st[i].mem_size:
                cnt[iset.names[ops[i * capi.MAX_GENOME + st[i].head[0] % st[i].mem_size]]] += 1
        o.step(0, n, budget=[1] * n, mode=capi.MODE_WORLD)
    tot = sum(cnt.values())
    for k, v in cnt.most_common():
        print("%-10s %6.2f%%" % (k, 100.0 * v / tot))


if __name__ == "__main__":
    main()
