"""Strip-tile overhead on one GPU (the multi-GPU cost
model): the bench-seeded world of X x Y cells run untiled, then as T row
strips through the halo protocol with the in-process loopback transport, both
after the same burn-in, K timed updates each (out == NULL: no statistics).
One GPU runs the T strips one after another on one stream, so

  per-strip update time   t_T = (time of one T-strip update) / T
  strip overhead          t_T - t_1 / T  (the strip's extra launches + copies)

and an update on T GPUs (one strip each) is predicted as t_T + the RCCL
exchange latencies the loopback copies stand for: an explicit term of
(dependent collective rounds per update, counted here) x (latency of one
small RCCL round over xGMI, AVGPU_RCCL_ROUND_US, default 20 us -- an assumed
figure: RCCL refuses two ranks on this pool's one GPU, so it is not measured
here) + the halo bytes at one xGMI link's ~50 GB/s.
usage (GPU box): python tools/strip_timing.py X Y T [burn_in] [K]   -> one JSON line"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import oracle_lib as ol
    from avida_amd import tiles
    from test_parity_full import _bench_seed, _seed
    X, Y, T = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 150
    K = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    golden = os.path.join(ROOT, "tests", "golden")
    cfg, iset, env, idx, gen, glen, gmer = _bench_seed(golden, X, Y)
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream)
    out = {"world": f"{X}x{Y}", "strips": T, "burn_in": B, "timed_updates": K}

    # untiled
    full = ol.Backend("gpu", cfg, iset, env, ncells=X * Y)
    full.lib.avgpu_set_stream(full.h, sp)
    _seed(full, 0, idx, gen, glen, gmer)
    for _ in range(B):
        full._call("run_update", full.h, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(K):
        full._call("run_update", full.h, None)
    torch.cuda.synchronize()
    t1 = (time.perf_counter() - t0) / K
    d_full = full.digests()
    full.close()
    del full
    print("untiled %.3f ms/update" % (t1 * 1e3), file=sys.stderr, flush=True)

    # T strips, loopback
    rows = Y // T
    strips = []
    for k in range(T):
        b = ol.Backend("gpu", cfg, iset, env, ncells=X * rows)
        b.lib.avgpu_set_stream(b.h, sp)
        t = tiles.Tile(b.lib, b.p, b.h, k * rows, T, "cuda")
        sl = slice(k * rows * X, (k + 1) * rows * X)
        _seed(b, 0, idx[sl], gen, glen, gmer)
        strips.append((b, t))
    class Counting(tiles.LoopbackTransport):
        """the loopback transport, counting the collective rounds"""
        rounds = 0

        def all_gather(self, tiles_):
            Counting.rounds += 1
            return super().all_gather(tiles_)

        def exchange(self, tiles_, kind):
            Counting.rounds += 1
            return super().exchange(tiles_, kind)

        def exchange_start(self, tiles_, kind):
            Counting.rounds += 1
            return super().exchange_start(tiles_, kind)

        def all_reduce_sum(self, tiles_):
            Counting.rounds += 1
            return super().all_reduce_sum(tiles_)

    world = tiles.StripWorld([t for _, t in strips], Counting())
    for _ in range(B):
        world.update()
    torch.cuda.synchronize()
    Counting.rounds = 0
    t0 = time.perf_counter()
    for _ in range(K):
        world.update()
    torch.cuda.synchronize()
    tT = (time.perf_counter() - t0) / K
    rounds = Counting.rounds / K
    rccl_us = float(os.environ.get("AVGPU_RCCL_ROUND_US", "20"))
    t0_ = strips[0][1]
    halo_bytes = 2 * (t0_.halo_send[0].numel() + t0_.rec_send[0].numel())
    comm_ms = rounds * rccl_us * 1e-3 + halo_bytes / 50e9 * 1e3
    import numpy as np
    d_strips = np.concatenate([b.digests() for b, _ in strips])
    out.update({
        "untiled_ms_per_update": round(t1 * 1e3, 4),
        "strips_ms_per_update": round(tT * 1e3, 4),
        "per_strip_ms": round(tT * 1e3 / T, 4),
        "ideal_per_strip_ms": round(t1 * 1e3 / T, 4),
        "strip_overhead_ms": round((tT - t1) * 1e3 / T, 4),
        "collective_rounds_per_update": rounds,
        "assumed_rccl_round_us": rccl_us,
        "predicted_ms_per_update_on_T_gpus": round(tT * 1e3 / T + comm_ms, 4),
        "predicted_weak_scaling_efficiency": round((t1 * 1e3 / T) / (tT * 1e3 / T + comm_ms), 3),
        "strips_equal_untiled": bool((d_full == d_strips).all()),
    })
    print(json.dumps(out))


if __name__ == "__main__":
    main()
