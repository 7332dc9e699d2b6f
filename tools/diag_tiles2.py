"""Diagnostic: oracle strips vs GPU strips, halo buffers compared after every
placement phase of every update (first difference printed)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch
import tile_util as tu
from avida_amd import tiles
g = os.path.join(ROOT, "tests", "golden")
X, Y, U, T = 64, 64, 13, 2
O = [tu.make_tile("oracle", g, X, Y, T, k) for k in range(T)]
G = [tu.make_tile("gpu", g, X, Y, T, k, device="cuda") for k in range(T)]
lo, lg = tiles.LoopbackTransport(), tiles.LoopbackTransport()
ot, gt = [t for _, t in O], [t for _, t in G]

def cmp(tag):
    torch.cuda.synchronize()
    for k in range(T):
        for d in range(2):
            a = ot[k].halo_send[d].numpy(); b = gt[k].halo_send[d].cpu().numpy()
            if (a != b).any():
                import numpy as np
                idx = np.nonzero(a != b)[0]
                print("DIFF", tag, "tile", k, "dir", d, "bytes", idx[:10], a[idx[:10]], b[idx[:10]], flush=True)
                return True
    return False

def both(f):
    f(ot, lo); f(gt, lg)

for u in range(U):
    for ts in (ot, gt):
        for t in ts: t.call("tile_partials", tiles.C.c_void_p(t.part.data_ptr()))
    lo.all_gather(ot); lg.all_gather(gt)
    for ts in (ot, gt):
        for t in ts: t.call("tile_begin", tiles.C.c_void_p(t.gathered.data_ptr()), T)
    if cmp(f"u{u} begin"): sys.exit(0)
    lo.exchange(ot, "halo"); lg.exchange(gt, "halo")
    for r in range(4):
        for ph in (0, 1):
            for ts in (ot, gt):
                for t in ts: t.call("tile_place", r, ph)
            if cmp(f"u{u} r{r} p{ph}"): sys.exit(0)
            lo.exchange(ot, "halo"); lg.exchange(gt, "halo")
        for ts in (ot, gt):
            for t in ts: t.call("tile_place", r, 2)
    for ts in (ot, gt):
        for t in ts: t.call("tile_place", 3, 3)
    torch.cuda.synchronize()
    for k in range(T):
        for d in range(2):
            a = ot[k].rec_send[d][:4].view(torch.int32)[0].item(); b = gt[k].rec_send[d][:4].cpu().view(torch.int32)[0].item()
            if a != b: print("REC COUNT DIFF u", u, k, d, a, b)
    lo.exchange(ot, "records"); lg.exchange(gt, "records")
    for ts in (ot, gt):
        for t in ts: t.call("tile_finish", None)
    torch.cuda.synchronize()
    so = [tu.tile_stats(b) for b, _ in O]; sg = [tu.tile_stats(b) for b, _ in G]
    print(u, [(s.births, s.births_dropped) for s in so], [(s.births, s.births_dropped) for s in sg], flush=True)
