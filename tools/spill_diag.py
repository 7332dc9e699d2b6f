"""Why class-0 slices spill (diagnostic; needs the SPD variant library built
with the spill counters 40-45): python tools/spill_diag.py"""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    from avida_amd import capi, files
    import bench
    lib = capi.load_product(os.path.join(ROOT, "avida_amd", "libavida_gpu_SPD.so"))
    h, cfg, n, _ = bench.build_world(lib, capi, files, os.path.join(ROOT, "tests", "golden"), 1024, 101, 0, 0, 1)
    for _ in range(150):
        capi.check(lib, lib.avgpu_run_update(h, None))
    tot = [0] * 6
    buf = (C.c_int64 * capi.NUM_COUNTERS)()
    for _ in range(20):
        capi.check(lib, lib.avgpu_run_update(h, None))
        capi.check(lib, lib.avgpu_counters(h, 0, buf, capi.NUM_COUNTERS))
        for k in range(6):
            tot[k] += buf[40 + k]
    print("per update: spills %.1f  after-divide %.1f  fresh %.1f  cur==blen %.1f  cur>blen %.1f  MAL %.1f"
          % tuple(x / 20 for x in tot))


if __name__ == "__main__":
    main()
