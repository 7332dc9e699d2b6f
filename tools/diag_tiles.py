"""Diagnostic: GPU single world vs oracle single world vs GPU strips on the
dense 64x64 tile-test world; prints the first update and cells that differ."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch
import tile_util as tu, parity_util as pu
from avida_amd import tiles
g = os.path.join(ROOT, "tests", "golden")
X, Y, U, T = 64, 64, 16, 2
CAP = 512
orc, _ = tu.single("oracle", g, X, Y, 0)
gpu, _ = tu.single("gpu", g, X, Y, 0)
pairs = [tu.make_tile("gpu", g, X, Y, T, k, device="cuda") for k in range(T)]
sw = tiles.StripWorld([t for _, t in pairs], tiles.LoopbackTransport())
def states(b, n):
    return b.states(0, n, CAP)
for u in range(U):
    so = orc.run_update(); sg = gpu.run_update(); sw.update(); torch.cuda.synchronize()
    st = [tu.tile_stats(b) for b, _ in pairs]
    print(u, "orc", so.insts_executed, so.births, "gpu", sg.insts_executed, sg.births,
          "tiles", sum(s.insts_executed for s in st), sum(s.births for s in st), flush=True)
    a = states(orc, X * Y); b = states(gpu, X * Y)
    bad = pu.diff_states(a[0], b[0], a[1], b[1], a[2], b[2], CAP)
    if bad:
        print("ORACLE vs GPU single differ at update", u, len(bad), bad[:6]); break
    per = X * Y // T
    for k, (tb, _) in enumerate(pairs):
        s = states(tb, per); lo = k * per
        bad = pu.diff_states(a[0][lo:lo + per], s[0], a[1][lo * CAP:(lo + per) * CAP], s[1],
                             a[2][lo * CAP:(lo + per) * CAP], s[2], CAP)
        if bad:
            print("ORACLE vs tile", k, "differ at update", u, len(bad), bad[:6]); sys.exit(0)
