"""Batch-vs-serial statistics of one world variant on spatial_res_100u
(diagnostic for DESIGN.md 4.3): the 60 trajectory KS tests, the 5 discovery
tests and the largest |d| per printed update, against the serial world
(cached in /tmp).

usage: python tools/piece_stats.py KIND [seeds] [ENV=VAL ...]
KIND: batchK / serial (tests/spatial_stats.py); ENV=VAL pairs are exported
before the workers start (oracle experiment knobs)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    kind = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    for kv in sys.argv[3:]:
        k, v = kv.split("=", 1)
        os.environ[k] = v
    import spatial_stats as ss
    cache = f"/tmp/serial_{n}.npz"
    if os.path.exists(cache):
        z = np.load(cache)
        s_tr, s_pr = z["tr"], z["pr"]
    elif kind == "serial":
        s_tr, s_pr = ss.runs("serial", n)
        np.savez(cache, tr=s_tr, pr=s_pr)
        return
    else:
        import subprocess
        env = {k: v for k, v in os.environ.items() if not k.startswith("ORACLE_")}
        subprocess.run([sys.executable, __file__, "serial", str(n)], env=env, check=True)
        z = np.load(cache)
        s_tr, s_pr = z["tr"], z["pr"]
    b_tr, b_pr = ss.runs(kind, n)
    tr = ss.trajectory_tests(b_pr, s_pr)
    di = ss.discovery_tests(b_tr, s_tr)
    thr = 0.01 / 65
    ps = sorted(tr + di, key=lambda x: x[1])
    print(f"{kind} {sys.argv[3:]} n={n}: min p {ps[0][1]:.3g} ({ps[0][0]}); failing {sum(p <= thr for _, p in ps)} / 65")
    d = np.abs(ss.effect_sizes(b_pr, s_pr))
    print("max |d| per printed update:", " ".join(f"{x:.2f}" for x in d.max(1)))
    mr = ss.mid_ranks(ss.reference(), b_pr)
    print(f"reference mid-rank range {mr.min():.4f}..{mr.max():.4f}")
    for name, p in ps[:5]:
        print(f"  {p:.3g}  {name}")


if __name__ == "__main__":
    main()
