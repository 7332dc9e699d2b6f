"""Per-phase clock breakdown of the class-0 interpreter launch (diagnostic).

Loads the AVGPU_PHASE_CLOCKS build (avida_amd/libavida_gpu_clk.so, built by
`python avida_amd/build.py --clocks`), runs the bench world for a few updates
and prints, per wave: s_memtime cycles spent staging (LDS-DMA of tapes +
stacks + state loads), in the interpreter loop, and writing back; loop
iterations (CNT_ITERS counts real loop iterations, parked lanes
included); and how many iterations entered the branch-free block, the h-copy
block and the switch (divergence: one iteration can enter several)."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (device init through HIP runtime in the library)
    from avida_amd import build, capi, files
    import bench
    side = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    updates = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    lib = capi.load_product(build.OUT_CLK)
    golden = os.path.join(ROOT, "tests", "golden")
    env_kind = sys.argv[4] if len(sys.argv) > 4 else "logic9"
    h, cfg, n, _ = bench.build_world(lib, capi, files, golden, side, 101, 0, 0, 1, env_kind=env_kind)
    burn = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    for _ in range(burn):
        capi.check(lib, lib.avgpu_run_update(h, None))
    tot = [0] * capi.NUM_COUNTERS
    buf = (C.c_int64 * capi.NUM_COUNTERS)()
    for _ in range(updates):
        capi.check(lib, lib.avgpu_run_update(h, None))
        capi.check(lib, lib.avgpu_counters(h, 0, buf, capi.NUM_COUNTERS))
        for k in range(capi.NUM_COUNTERS):
            tot[k] += buf[k]
    waves = max(1, tot[capi.CNT_WAVES])
    it = max(1, tot[capi.CNT_ITERS])
    out = {
        "side": side, "env": env_kind, "updates": updates, "waves_per_update": waves / updates,
        "stage_cycles_per_wave": tot[capi.CNT_CLK_STAGE] / waves,
        "loop_cycles_per_wave": tot[capi.CNT_CLK_LOOP] / waves,
        "wb_cycles_per_wave": tot[capi.CNT_CLK_WB] / waves,
        "iters_per_wave": it / waves,
        "loop_cycles_per_iter": tot[capi.CNT_CLK_LOOP] / it,
        "frac_iters_fast": tot[capi.CNT_IT_FAST] / it,
        "frac_iters_copy": tot[capi.CNT_IT_COPY] / it,
        "frac_iters_slow": tot[capi.CNT_IT_SLOW] / it,
        "c0_slices_per_update": tot[capi.CNT_C0_SLICES] / updates,
        "c0_sites_per_slice": tot[capi.CNT_C0_SITES] / max(1, tot[capi.CNT_C0_SLICES]),
        "lane_efficiency": tot[capi.CNT_INSTS] / max(1, tot[capi.CNT_LANESTEPS]),
        "spills_per_update": tot[capi.CNT_SPILLS] / updates,
        "loop_cycles_per_iter_by_block": {k: tot[32 + i] / it for i, k in enumerate(
            ["decode", "fast", "copy", "switch", "wave_phase", "advance"])},
        "slow_phase_cycles_per_iter_by_case": {k: tot[38 + i] / it for i, k in enumerate(
            ["pop", "push", "io", "h_alloc", "h_divide", "h_search", "if_label", "pre_switch",
             "io2_task_lookup", "io2_rewards"])},
    }
    lib.avgpu_destroy(h)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
