"""Batch steps per update of the product world (diagnostic for DESIGN.md
4.2): the oracle's batch world seeded like bench.py (detail-50000.pop, loaded
in lock step) with the logic-9 or configs[4] resource environment, its
adaptive K (avgpu_update_stats.sub_steps) and predictor per update.

usage: python tools/k_study.py logic9|resources SIDE UPDATES"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import bench
    from avida_amd import capi, files
    import oracle_lib as ol
    kind, side, upd = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    golden = os.path.join(ROOT, "tests", "golden")
    iset, pool = bench._pool(golden)
    env = bench.environment(files, golden, kind, side, side)
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None, {"WORLD_X": side, "WORLD_Y": side}), seed=101)
    n = side * side
    b = ol.Backend("oracle", cfg, iset, env, ncells=n)
    picks = bench._genomes_for(n, pool)
    b.set_orgs(0, [g for g, _ in picks], merits=[m for _, m in picks], deterministic=False)
    ks, ds, es = [], [], []
    for _ in range(upd):
        st = b.run_update()
        ks.append(st.sub_steps)
        ds.append(st.sched_pred_cnt / max(1, st.sched_pred_n))
        es.append(abs(st.sched_pred) / 1048576 / max(1, st.sched_pred_n))
    ks = np.array(ks)
    print(f"{kind} {side}x{side}: K per 10 updates", [round(float(ks[i:i + 10].mean()), 2) for i in range(0, upd, 10)])
    print(f"last 50 updates: K {ks[-50:].mean():.2f}, densest-quarter D {np.mean(ds[-50:]):.3f}, "
          f"weight E {np.mean(es[-50:]):.3f}")


if __name__ == "__main__":
    main()
