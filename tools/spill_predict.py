"""Which organisms spill out of class 0, and could the allotment see it
coming?  (diagnostic, CPU only: runs the oracle's batch world, whose
updates are the GPU's bit for bit)

A class-0 slice spills when an h-alloc would grow the memory past
CLASS0_SIZE; the slice then ends in the spill row after class 0, so from the
end-of-update state: need_of(start) <= 320 and memory(end) > 320.  For those
organisms and for all other class-0 slices this prints the read head at the
start of the update, to test "read head > CLASS0_SIZE / 3" as a predictor.

  python tools/spill_predict.py [side] [burn] [updates]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def need_of(m, mal):
    return m if mal else m + min(2 * m, 2048 - m)


def main():
    from avida_amd import capi, files
    import bench
    from oracle_lib import Backend, GOLDEN
    side = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    burn = int(sys.argv[2]) if len(sys.argv) > 2 else 150
    ups = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    iset, pool = bench._pool(GOLDEN)
    env = bench.environment(files, GOLDEN, "logic9", side, side)
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None, {"WORLD_X": side, "WORLD_Y": side}), seed=101)
    b = Backend("oracle", cfg, iset, env)
    n = side * side
    picks = bench._genomes_for(n, pool)
    b.set_orgs_np(0, b"".join(g for g, _ in picks), np.array([len(g) for g, _ in picks]),
                  np.array([m for _, m in picks]))
    for _ in range(burn):
        b.run_update()
    spilled, quiet = [], []
    for _ in range(ups):
        st0, _, _ = b.states(0, n, cap=1)
        b.run_update()
        st1, _, _ = b.states(0, n, cap=1)
        for c in range(n):
            s0, s1 = st0[c], st1[c]
            if not (s0.alive and s1.alive) or s1.birth_length != s0.birth_length:
                continue
            if need_of(s0.mem_size, s0.mal_active) > 320:
                continue
            rec = (s0.head[1], s0.mem_size, s0.mal_active, s0.birth_length, s1.mem_size)
            (spilled if s1.mem_size > 320 else quiet).append(rec)
    sp, qu = np.array(spilled).reshape(-1, 5), np.array(quiet).reshape(-1, 5)
    print(f"{ups} updates of a {side}x{side} world after {burn}: class-0 slices {len(sp) + len(qu)}, "
          f"spilled {len(sp)} ({len(sp) / ups:.1f} per update)")
    for thr in (100, 104, 108, 112):
        print(f"  read head > {thr} at start: spilled {np.mean(sp[:, 0] > thr) if len(sp) else 0:.2f}, "
              f"others {np.mean(qu[:, 0] > thr):.4f} ({int(np.sum(qu[:, 0] > thr))})")
    if len(sp):
        print("  spilled (rh, mem, mal, birth_len, mem_end) first 20:", sp[:20].tolist())


if __name__ == "__main__":
    main()
