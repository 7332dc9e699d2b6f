"""Diagnostic: BIRTH_METHOD 4 at the bench's world size -- a 1024 x 1024 grid
seeded with 256 ancestor mutants, 40 batch updates, GPU == oracle counters
every update and every digest at the end."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as ol  # noqa: E402
import parity_util as pu  # noqa: E402
from avida_amd import files  # noqa: E402

golden = os.path.join(ROOT, "tests", "golden")
ov = {"WORLD_X": 1024, "WORLD_Y": 1024, "BIRTH_METHOD": 4}
iset, env, cfg = pu.load_env(golden, overrides=ov, seed=11)
n = cfg.world_x * cfg.world_y
anc = files.read_org(os.path.join(golden, "default-heads.org"), iset)
g = pu.mutants_of(anc, iset, 256, rate=0.02, seed=9)
orc = ol.Backend("oracle", cfg, iset, env, ncells=n)
gpu = ol.Backend("gpu", cfg, iset, env, ncells=n)
for b in (orc, gpu):
    b.set_orgs(0, g, deterministic=False)
for u in range(40):
    so, sg = orc.run_update(), gpu.run_update()
    a = (so.num_organisms, so.births, so.insts_executed)
    b = (sg.num_organisms, sg.births, sg.insts_executed)
    print(u, a, b, flush=True)
    assert a == b
nbad, cells = pu.compare_digests(orc.digests(), gpu.digests())
print("digest mismatches", nbad)
assert nbad == 0
