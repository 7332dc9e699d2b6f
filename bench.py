"""Throughput benchmark of the batched heads-CPU interpreter (one JSON line).

Workload (BASELINE.json configs[2], metric "organism-instructions/sec +
updates/sec, 1M-org logic-9 world"): a 1024x1024 torus per GPU, logic-9
environment, default avida.cfg mutation rates (copy 0.0075, divide ins/del
0.05), births on.  Every cell starts occupied by an evolved logic-9 genotype
from the reference's own fixture (tests/heads_midrun_30u/config/
detail-50000.pop, classic legacy instset; inputs synthetic per cell), so the
timed updates measure a mature population rather than an ancestor ramp-up.

A "step" is one whole Avida update (Avida2Driver::Run loop body): merit-
weighted allotment of AVE_TIME_SLICE*N instructions, interpretation, birth
placement, statistics.  value = organism-instructions executed by all ranks /
max-over-ranks wall time of the K timed updates.

Multi-GPU (torch.distributed.run, one rank per GPU, RCCL over xGMI): the
world is ONE 1024 x (1024*N) torus cut into N row strips of 1024x1024 (weak
scaling).  Every update all-gathers the 256-cell merit partials (the
scheduler's global total, cMultiProcessWorld.cc:375-405) and exchanges
occupancy / placement claims / offspring across strip edges
(avida_amd/tiles.py), so the N-GPU run is cell for cell the untiled world.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "organism-instructions/sec + updates/sec, 1M-org logic-9 world, 1/8 GPUs"
# SURVEY.md 8(d) algorithmic bytes: per organism time slice the packed
# architectural + phenotype state (224 B) is read and written, and the memory
# tape at 1.25 B/site (op byte + 2 flag bits) is read and written.
STATE_BYTES = 224.0
SITE_BYTES = 1.25
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md chip table (spec)
# updates run before the timed region (+ the warmup): the timed world is aged,
# not the freshly seeded lock-step one (tests/test_parity_full.py checks parity
# in exactly this regime)
BURN_IN = 150
WARMUP = 5
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_k_interpret320.json")



def issue_roofline(cnt, c0_ms, c0_insts):
    """Instruction-issue roofline of k_interpret<320> (the second roofline the
    north star asks for). PMC wave-instruction counts per class-0 dispatch
    (profiles/pmc_k_interpret320.json, same world) over this run's live
    HIP-event duration of that kernel. VALU peak: a wave64 VALU instruction
    occupies its SIMD-32 for 2 cycles (MI355X_MICROARCH.md, wave scheduling),
    4 SIMDs x 256 CUs x 2.4 GHz / 2 = 1.23e12 wave-instructions/s; SALU peak:
    one scalar instruction per CU per cycle = 6.1e11/s. `oi_ceiling` is the
    OI/s at which VALU issue alone would saturate with this build's VALU
    instructions per organism instruction."""
    if c0_ms <= 0 or c0_insts <= 0:
        return None
    sec = c0_ms * 1e-3
    valu, salu = cnt["SQ_INSTS_VALU"], cnt["SQ_INSTS_SALU"]
    valu_peak = 256 * 4 * 2.4e9 / 2.0
    salu_peak = 256 * 2.4e9
    wc = cnt["SQ_WAVE_CYCLES"]
    return {
        "bound": "valu-issue",
        "achieved": valu / sec,
        "peak": valu_peak,
        "unit": "wave-instructions/s",
        "frac": valu / sec / valu_peak,
        "salu_frac": salu / sec / salu_peak,
        "valu_per_oi": valu / c0_insts,
        "oi_ceiling": valu_peak / (valu / c0_insts),
        "wave_cycles_active": cnt["SQ_ACTIVE_INST_ANY"] / wc,
        "wave_cycles_waitcnt": cnt["SQ_WAIT_ANY"] / wc,
        "wave_cycles_issue_stall": cnt["SQ_WAIT_INST_ANY"] / wc,
        "lds_bank_conflict_frac": cnt["SQ_LDS_BANK_CONFLICT"] / max(1.0, cnt["SQ_LDS_IDX_ACTIVE"]),
    }
def _pool(golden):
    from avida_amd import files
    iset = files.read_instset(os.path.join(golden, "instset-classic.cfg"))
    pool = []
    for g in files.read_pop(os.path.join(golden, "detail-50000.pop")):
        # cPopulation::LoadPopulation keeps the recorded merit (main/cPopulation.cc:6723-7000)
        pool.extend([(iset.parse_sequence(g.sequence), g.merit)] * g.num_cpus)
    return iset, pool


def _genomes_for(n, pool, first=0):
    """genotype of global cells first .. first+n-1 (a fixed hash of the cell id)"""
    import numpy as np
    idx = ((np.arange(n, dtype=np.uint64) + np.uint64(first)) * np.uint64(2654435761)) % np.uint64(len(pool))
    return [pool[int(i)] for i in idx]


LOGIC9 = [("NOT", "not", 1.0), ("NAND", "nand", 1.0), ("AND", "and", 2.0), ("ORN", "orn", 2.0),
          ("OR", "or", 4.0), ("ANDN", "andn", 4.0), ("NOR", "nor", 8.0), ("XOR", "xor", 8.0),
          ("EQU", "equ", 16.0)]


def resource_env_text(X, Y, inflow_per_cell=1.0, outflow=0.01):
    """configs[4]: resource-limited logic-9 -- one spatial torus resource per
    reaction, inflow and outflow over the whole world, diffusion on; the
    reactions follow the reference's resources_9r environment (frac=0.0025,
    max=25, additive bonus consumed * value, values 1 1 2 2 4 4 8 8 16)"""
    box = f"inflowx1=0:inflowx2={X - 1}:inflowy1=0:inflowy2={Y - 1}:" \
          f"outflowx1=0:outflowx2={X - 1}:outflowy1=0:outflowy2={Y - 1}"
    lines = [f"RESOURCE res{name}:geometry=torus:initial={X * Y * inflow_per_cell}:"
             f"inflow={X * Y * inflow_per_cell}:outflow={outflow}:{box}:xdiffuse=1:ydiffuse=1"
             for name, _, _ in LOGIC9]
    lines += [f"REACTION {name} {task} process:resource=res{name}:value={v}:frac=0.0025:max=25"
              for name, task, v in LOGIC9]
    return "\n".join(lines) + "\n"


def environment(files, golden, kind, X, Y):
    if kind == "resources":
        return files.parse_environment(resource_env_text(X, Y))
    return files.read_environment(os.path.join(golden, "environment-logic9.cfg"))


def build_world(lib, capi, files, golden, side, seed, device, rank, world, on_tile=None, env_kind="logic9",
                sub_updates=0):
    """One 1024x1024 strip per rank of a side x (side*world) torus (world = 1:
    the untiled side x side world).  on_tile(h) places the strip before the
    organisms are injected (their RNG streams are keyed by global cell id)."""
    iset, pool = _pool(golden)
    env = environment(files, golden, env_kind, side, side * world)
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None, {"WORLD_X": side, "WORLD_Y": side * world}),
                              seed=seed)
    cfg.sub_updates = sub_updates
    n = side * side
    h = lib.avgpu_create(C.byref(cfg), device, n)
    if not h:
        raise RuntimeError(lib.avgpu_last_error().decode())
    hid = (C.c_uint8 * len(iset.names))(*iset.handlers)
    red = (C.c_int32 * len(iset.names))(*iset.redundancy)
    capi.check(lib, lib.avgpu_load_instset(h, len(iset.names), hid, red))
    if env.resources:
        ra, ca = capi.resources_arrays(env.resources, env.cells)
        capi.check(lib, lib.avgpu_load_resources(h, len(env.resources), ra, len(env.cells), ca))
    arr = capi.reactions_array(env)
    capi.check(lib, lib.avgpu_load_env(h, len(env), arr))
    tile = on_tile(h) if on_tile else None
    picks = _genomes_for(n, pool, rank * n)
    blob = b"".join(g for g, _ in picks)
    buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
    lens = (C.c_int32 * n)(*[len(g) for g, _ in picks])
    merits = (C.c_double * n)(*[m for _, m in picks])
    capi.check(lib, lib.avgpu_set_orgs(h, 0, n, buf, lens, merits, None, 0))
    return h, cfg, n, tile


def cpu_baseline(golden, seconds, env_kind="logic9"):
    """Reference-style serial world (tests/oracle_lib.py, CPU restatement) on one
    host core: a 60x60 world filled from the same genotype pool, updates until
    `seconds` elapse."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from avida_amd import capi, files
    import oracle_lib as ol
    iset, pool = _pool(golden)
    env = environment(files, golden, env_kind, 60, 60)
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None), seed=101)
    n = cfg.world_x * cfg.world_y
    b = ol.Backend("oracle", cfg, iset, env, ncells=n)
    picks = _genomes_for(n, pool)
    b.set_orgs(0, [g for g, _ in picks], merits=[m for _, m in picks], deterministic=False)
    st = capi.AvgpuUpdateStats()
    updates = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        b.lib.orc_run_serial_updates(b.h, 10, C.byref(st))
        updates += 10
    dt = time.perf_counter() - t0
    insts = st.cum_insts_executed
    return {"value": insts / dt, "unit": "organism-instructions/s", "cores": 1, "kind": "port",
            "sample": f"oracle serial world (reference-style scheduler + speculative steps), "
                      f"60x60 evolved logic-9 population ({env_kind} environment), {updates} updates, {insts} insts, "
                      f"{dt:.1f} s on 1 host core",
            "updates_per_sec": updates / dt}


def cpu_baseline_multi(golden, seconds, env_kind, procs):
    """the reference's rate_runner measures P independent
    processes, one per host core, and sums their OI/s.  Each worker is a
    fresh `python bench.py --cpu-worker` child (started before this process
    touches the GPU) running the single-core baseline for `seconds`."""
    import subprocess
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-worker", "--cpu-seconds", str(seconds),
           "--env", env_kind]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    ps = [subprocess.Popen(cmd, stdout=subprocess.PIPE, env=env) for _ in range(procs)]
    outs = [json.loads(p.communicate()[0].decode().strip().splitlines()[-1]) for p in ps]
    if any(p.returncode for p in ps):
        raise RuntimeError("a CPU baseline worker failed")
    single = outs[0]
    return {"value": sum(o["value"] for o in outs), "unit": "organism-instructions/s", "cores": procs,
            "kind": "port", "single_core_value": single["value"],
            "host_cpus": os.cpu_count(),
            # the box gives one GPU's job a share of 16 host CPUs (gpurun's
            # worker-pool rule); the whole host, linearly extrapolated from the
            # single-core rate (independent worlds share nothing; an upper bound)
            "all_host_cpus_extrapolated": single["value"] * (os.cpu_count() or 1),
            "label": "restatement (reference unbuildable here: its libs/apto submodule is absent)",
            "sample": f"{procs} independent oracle serial worlds (one process per host core, like the "
                      f"reference's heads_perf_1000u_rate rate_runner; {procs} of the box's "
                      f"{os.cpu_count()} host CPUs), each: {single['sample']}",
            "updates_per_sec": sum(o["updates_per_sec"] for o in outs)}


def free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch_ranks(n, argv, script=None, env=None):
    """`bench.py --gpus N` started without torch.distributed.run (no
    WORLD_SIZE in the environment): this parent process -- which has not
    touched the GPU -- starts the N ranks itself, one per GPU, exactly as the
    driver's multi-GPU form does (python -m torch.distributed.run --nnodes=1
    --nproc-per-node N --master-addr 127.0.0.1 ...), and exits with their
    status.  Rank 0 prints the JSON line.  (cMultiProcessWorld,
    main/cMultiProcessWorld.cc:375-405, is the reference's multi-process
    world; here one process per GPU, RCCL over xGMI.)"""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}",
           script or os.path.abspath(__file__)] + list(argv)
    return subprocess.run(cmd, env=env).returncode


def rank_env(gpus):
    """(rank, world, local rank) of this process; under torch.distributed.run
    WORLD_SIZE must equal --gpus, so that n_gpus in the JSON line is what ran."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if "WORLD_SIZE" in os.environ and world != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {gpus}")
    return rank, world, local


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--side", type=int, default=1024)
    ap.add_argument("--burn-in", type=int, default=BURN_IN,
                    help="untimed updates that age the seeded population before the warmup "
                         "(its organisms start in lock step; ~10 gestations spread them out)")
    ap.add_argument("--seed", type=int, default=101)
    ap.add_argument("--time-every", type=int, default=4,
                    help="bracket every k-th update's class-0 launch with HIP events (roofline timing; "
                         "each event record leaves a few us of dead time on the stream)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--env", choices=["logic9", "resources"], default="logic9",
                    help="logic9: configs[2] (the metric's workload); resources: configs[4], "
                         "one diffusing spatial resource per logic-9 reaction")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="CPU baseline processes (0: min(16, host CPUs) -- 16 is a GPU box's share)")
    ap.add_argument("--cpu-worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--sub-updates", type=int, default=0,
                    help="batch steps per update (avgpu_cfg.sub_updates, DESIGN.md 4.2): 0 is the "
                         "product's default (adaptive: more steps in an update whose total weight "
                         "is expected to move); K > 0 always K steps")
    ap.add_argument("--long-updates", type=int, default=200,
                    help="after the K timed steps, a second untimed-by-contract run of this many "
                         "updates reported as config.long_run (stability cross-check; 0 = off)")
    args = ap.parse_args()
    golden = os.path.join(ROOT, "tests", "golden")
    if args.cpu_worker:                       # one CPU baseline process (no GPU)
        print(json.dumps(cpu_baseline(golden, args.cpu_seconds, args.env)), flush=True)
        return
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_ranks(args.gpus, sys.argv[1:]))
    rank, world, local = rank_env(args.gpus)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:   # before this process initialises the GPU
        procs = args.cpu_procs or min(16, os.cpu_count() or 1)
        cpu = cpu_baseline_multi(golden, args.cpu_seconds, args.env, procs)

    import torch
    # AVGPU_BENCH_STAGED=1: a rehearsal of the multi-GPU bench on fewer GPUs --
    # ranks may share a device, exchanges over gloo staged through host
    # tensors (tiles.StagedTransport; RCCL refuses two ranks on one device).
    # Its line says so in config.transport and is no scaling measurement.
    staged = os.environ.get("AVGPU_BENCH_STAGED") == "1" and world > 1
    rdev = "cpu" if staged else "cuda"      # the timing / counter reductions' tensors
    device = local % max(1, torch.cuda.device_count()) if staged else local
    torch.cuda.set_device(device)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo" if staged else "nccl")
        assert dist.get_world_size() == world == args.gpus

    from avida_amd import capi, files, tiles
    lib = capi.load_product()
    golden = os.path.join(ROOT, "tests", "golden")
    stream = torch.cuda.current_stream()

    def on_tile(h):
        capi.check(lib, lib.avgpu_set_stream(h, C.c_void_p(stream.cuda_stream)))
        if world == 1:
            return None
        return tiles.Tile(lib, "avgpu_", h, rank * args.side, world, "cuda")

    h, cfg, n, tile = build_world(lib, capi, files, golden, args.side, args.seed, device, rank, world,
                                  on_tile, args.env, args.sub_updates)
    transport = (tiles.StagedTransport(dist) if staged else tiles.DistTransport(dist)) if tile else None
    strips = tiles.StripWorld([tile], transport) if tile else None

    capi.check(lib, lib.avgpu_set_timing(h, args.time_every))

    def ref_insts():
        """cumulative organism-instructions of the reference's semantics:
        executed, less those replaced organisms ran after their newborns'
        births"""
        st = capi.AvgpuUpdateStats()
        capi.check(lib, lib.avgpu_get_stats(h, C.byref(st)))
        cnt = (C.c_int64 * capi.NUM_COUNTERS)()
        capi.check(lib, lib.avgpu_counters(h, 1, cnt, capi.NUM_COUNTERS))
        return st.cum_insts_executed - cnt[capi.CNT_WASTED]

    def update():
        if strips:
            strips.update()      # halo-birth exchange + gathered scheduler totals over RCCL
        else:
            capi.check(lib, lib.avgpu_run_update(h, None))

    for _ in range(args.burn_in + args.warmup):
        update()
    torch.cuda.synchronize()
    s0 = capi.AvgpuUpdateStats()
    capi.check(lib, lib.avgpu_get_stats(h, C.byref(s0)))
    cms, phases = (C.c_double * 4)(), C.c_int64()
    capi.check(lib, lib.avgpu_kernel_times(h, cms, C.byref(phases)))  # reset
    cnt0 = (C.c_int64 * capi.NUM_COUNTERS)()
    capi.check(lib, lib.avgpu_counters(h, 1, cnt0, capi.NUM_COUNTERS))

    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        update()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()

    s1 = capi.AvgpuUpdateStats()
    capi.check(lib, lib.avgpu_get_stats(h, C.byref(s1)))
    capi.check(lib, lib.avgpu_kernel_times(h, cms, C.byref(phases)))
    cnt1 = (C.c_int64 * capi.NUM_COUNTERS)()
    capi.check(lib, lib.avgpu_counters(h, 1, cnt1, capi.NUM_COUNTERS))
    d = [cnt1[k] - cnt0[k] for k in range(capi.NUM_COUNTERS)]
    # the organism-instructions of the reference's semantics: every executed
    # instruction (main pass + newborn pass) but those an organism ran after
    # the birth of the offspring that replaced it
    insts = (s1.cum_insts_executed - s0.cum_insts_executed) - d[capi.CNT_WASTED]
    births = s1.cum_births - s0.cum_births
    dt = t1 - t0
    vec = torch.tensor([dt, float(insts), float(births), float(s1.num_organisms)],
                       dtype=torch.float64, device=rdev)
    if dist:
        mx = vec.clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(vec)
        dt_max = mx[0].item()
    else:
        dt_max = vec[0].item()
    tot_insts, tot_births, tot_orgs = vec[1].item(), vec[2].item(), vec[3].item()
    nph = max(1, phases.value)
    # offspring never placed (birth-queue overflow, oversize, full halo arena:
    # placement itself places every birth), offspring placed and then
    # overwritten by a later birth into the same cell, and slices handed to a
    # larger LDS class, summed over ranks
    extra = torch.tensor([float(d[capi.CNT_DROPPED]), float(d[capi.CNT_SPILLS]),
                          float(d[capi.CNT_OVERWRITTEN]), float(d[capi.CNT_WASTED])],
                         dtype=torch.float64, device=rdev)
    if dist:
        dist.all_reduce(extra)
    long_run = None
    if args.long_updates > 0:
        # stability cross-check outside the contract's timed region: the same
        # updates, many more of them, under the same barrier / max-over-ranks clock
        li0 = ref_insts()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        l0 = time.perf_counter()
        for _ in range(args.long_updates):
            update()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        ldt = torch.tensor([time.perf_counter() - l0], dtype=torch.float64, device=rdev)
        lins = torch.tensor([float(ref_insts() - li0)],
                            dtype=torch.float64, device=rdev)
        if dist:
            dist.all_reduce(ldt, op=dist.ReduceOp.MAX)
            dist.all_reduce(lins)
        long_run = {"updates": args.long_updates, "value": lins.item() / ldt.item(),
                    "ms_per_step": ldt.item() * 1e3 / args.long_updates}
    stats_run = None
    if args.long_updates > 0 and world == 1:
        # the timed updates skip the statistics reduction the reference runs
        # every update (cPopulation::UpdateOrganismStats, main/cPopulation.cc:6245;
        # DESIGN.md 5 "lazy statistics"): the same updates with it, stream-ordered
        # (avgpu_stats_vector enqueues the reduction, no host copy)
        # (its cost: 20 updates without it, then 20 with it, back to back, so
        # that the population's drift since the timed region cancels)
        nst = 20
        si0 = ref_insts()
        ptr = C.c_void_p()
        torch.cuda.synchronize()
        p0 = time.perf_counter()
        for _ in range(nst):
            update()
        torch.cuda.synchronize()
        pdt = time.perf_counter() - p0
        q0 = time.perf_counter()
        for _ in range(nst):
            update()
            capi.check(lib, lib.avgpu_stats_vector(h, C.byref(ptr)))
        torch.cuda.synchronize()
        qdt = time.perf_counter() - q0
        stats_run = {"updates": nst, "value": (ref_insts() - si0) / (pdt + qdt),
                     "ms_per_step": qdt * 1e3 / nst, "ms_per_step_without": pdt * 1e3 / nst,
                     "stats_ms_per_update": (qdt - pdt) * 1e3 / nst}
    if rank != 0:
        if dist:
            dist.destroy_process_group()
        return
    value = tot_insts / dt_max
    # roofline of the dominant kernel k_interpret<320> (LDS size class 0, one
    # launch per update), this rank: algorithmic bytes per launch =
    # slices * 2 * 224 B + tape sites staged in and written back * 1.25 B,
    # over its HIP-event-timed average duration on the world's stream.
    c0_ms = cms[0] / nph
    # counters run over every update of the timed region (one class-0 launch
    # per batch step -- the newborn pass's is not counted); the events only
    # over every time_every-th launch
    launches = max(1, d[capi.CNT_STEPS])
    c0_slices = d[capi.CNT_C0_SLICES] / launches
    c0_sites = d[capi.CNT_C0_SITES] / launches
    bytes_per_launch = 2.0 * STATE_BYTES * c0_slices + SITE_BYTES * c0_sites
    achieved = bytes_per_launch / (c0_ms * 1e-3) / 1e9 if c0_ms > 0 else 0.0
    traffic, traffic_src, issue = None, None, None
    if os.path.exists(PMC_FILE):
        with open(PMC_FILE) as f:
            pmc = json.load(f)
        same_build = pmc.get("lib_sha16") == capi.lib_build_hash()
        if pmc.get("world") == f"{args.side}x{args.side}" and args.env == "logic9":
            if same_build:
                traffic = pmc["hbm_bytes_per_launch"]
                traffic_src = pmc["source"]
                issue = issue_roofline(pmc["counters_per_dispatch"], c0_ms,
                                       d[capi.CNT_INSTS] / args.steps * c0_slices /
                                       max(1.0, d[capi.CNT_SLICES] / args.steps))
            else:     # counters of another build of the library: not paired with this run's timing
                traffic_src = (f"none: {PMC_FILE} holds counters of library build {pmc.get('lib_sha16')}, "
                               f"this is {capi.lib_build_hash()} (rerun tools/pmc_passes.sh)")
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "organism-instructions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt_max * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {
            "workload": (f"configs[2]: {args.side}x{args.side} torus per GPU, logic-9, default "
                         "avida.cfg mutation rates, births on, seeded with the detail-50000.pop "
                         "evolved genotypes (classic instset)") if args.env == "logic9" else
                        (f"configs[4]: {args.side}x{args.side} torus per GPU, resource-limited logic-9 "
                         "(9 spatial torus resources, inflow/outflow everywhere, diffusion 1), default "
                         "mutation rates, births on, seeded with the detail-50000.pop genotypes"),
            "environment": args.env,
            "world": f"{args.side}x{args.side}x{world}",
            "burn_in_updates": args.burn_in,
            "organisms": int(tot_orgs),
            "updates_per_sec": args.steps / dt_max,
            "births_per_update": tot_births / args.steps,
            "births_never_placed_per_update": extra[0].item() / args.steps,
            "births_overwritten_per_update": extra[2].item() / args.steps,
            "spills_per_update": extra[1].item() / args.steps,
            "insts_per_update": tot_insts / args.steps,
            "insts_wasted_per_update": extra[3].item() / args.steps,
            "parallelism": f"strips{world}",
            "transport": ("gloo-staged rehearsal (ranks share GPUs; not a scaling measurement)" if staged
                          else ("rccl" if world > 1 else "none")),
            "ranks": world,
            "sub_updates": args.sub_updates,
            "batch_steps_per_update": d[capi.CNT_STEPS] / args.steps,
            "long_run": long_run,
            # the timed updates run without the per-update statistics reduction;
            # stats_every_update_run: the same updates with it (its cost per update)
            "stats_every_update": False,
            "stats_every_update_run": stats_run,
        },
        # The resource that binds k_interpret<320> is instruction issue plus
        # exposed latency, so the headline roofline is the VALU-issue one
        # (PMC wave-instructions per launch over the live event-timed launch);
        # the HBM roofline of the same launch (algorithmic bytes of SURVEY.md
        # 8(d) over the same duration, PMC traffic) follows as "hbm".
        "roofline": {
            "bound": "issue",
            "binding": "VALU instruction issue + exposed LDS / memory latency",
            "achieved": issue["achieved"] if issue else None,
            "peak": issue["peak"] if issue else None,
            "unit": "wave-instructions/s",
            "frac": issue["frac"] if issue else None,
            "traffic": traffic,
            "traffic_source": traffic_src,
            "hbm": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                    "traffic_over_algorithmic": (traffic / bytes_per_launch) if traffic else None},
            "kernel": "k_interpret<320> (LDS size class 0)",
            "kernel_ms": c0_ms,
            "timed_launches": int(phases.value),
            "time_every": args.time_every,
            "bytes_per_launch": bytes_per_launch,
            "slices_per_launch": c0_slices,
            "mean_sites_per_slice": c0_sites / max(1.0, 2.0 * c0_slices),
            "all_classes_ms": sum(cms) / nph,
            "class_ms": [x / nph for x in cms],
            "lane_efficiency": d[capi.CNT_INSTS] / max(1, d[capi.CNT_LANESTEPS]),
            "insts_per_kernel_second": d[capi.CNT_INSTS] / max(1e-9, sum(cms) * 1e-3),
            "issue": issue,
        },
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu
    lib.avgpu_destroy(h)
    print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
