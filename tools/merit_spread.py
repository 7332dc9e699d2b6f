"""The bench world's merit spread (diagnostic for DESIGN.md 8, the newborn
pass): after the bench's burn-in, the quantiles of merit / mean merit over the
living organisms -- a slice's expected budget is AVE_TIME_SLICE x that ratio,
and a newborn's share of its birth step (1 - t) of it, so the largest ratios
set the longest waves of the main and the newborn pass.

usage (GPU box): python tools/merit_spread.py [updates]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from avida_amd import capi, files
    upd = int(sys.argv[1]) if len(sys.argv) > 1 else 160
    lib = capi.load_product()
    golden = os.path.join(ROOT, "tests", "golden")
    h, cfg, n, _ = bench.build_world(lib, capi, files, golden, 1024, 1, 0, 0, 1)
    for _ in range(upd):
        capi.check(lib, lib.avgpu_run_update(h, None))
    cen = capi.get_census(lib, "avgpu_", h, 0, n)
    st = capi.AvgpuUpdateStats()
    capi.check(lib, lib.avgpu_get_stats(h, C.byref(st)))
    m = cen["merit"][cen["genome_length"] > 0]
    r = m / m.mean()
    qs = [0.5, 0.9, 0.99, 0.999, 0.9999, 1.0]
    print(f"organisms {st.num_organisms}, births {st.births}, mean merit {m.mean():.1f}")
    print("merit / mean at quantiles " + "  ".join(f"{q}: {np.quantile(r, q):.2f}" for q in qs))
    print(f"expected slice budget of the top organism {cfg.ave_time_slice * r.max():.0f} instructions")
    lib.avgpu_destroy(h)


if __name__ == "__main__":
    main()
