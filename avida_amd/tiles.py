"""Host driver of strip-tiled worlds: one global Avida world split into row
strips, one strip per GPU (or several strips in one process for tests).

This is the host half of the multi-GPU row of the hot path.  It
replaces cMultiProcessWorld (main/cMultiProcessWorld.cc:142-190 migrant
exchange, :375-405 update-size all-reduce) -- the reference's only
multi-process world -- with strips of ONE torus, so that an update of the
tiled world equals the same update of the untiled world cell for cell
(DESIGN.md "Multi-GPU").  The per-update schedule is the one documented in
include/avida_gpu.h ("strip tiles"):

    tile_partials -> all_gather -> tile_steps (K) -> per batch step s < K:
    [s > 0: tile_partials -> all_gather] -> tile_begin_step -> exchange(halo)
    tile_place(0, 0) (picks, kill times) -> exchange(halo)
    tile_place(0, 3) (cancellations, round-0 claims) -> exchange(halo)
    3 x [tile_place(r, 0) -> exchange(halo)]
    tile_place(3, 1) -> exchange(records) issued -> tile_place(3, 2) (own
    winners, while the records travel) -> wait(records) -> tile_finish
    with resources: exchange(resources) after the all_gather (edge rows of
    the spatial grids), all_reduce(consumption) + tile_res_settle at the end

`lib` may be the product (prefix "avgpu_", device buffers, RCCL/NCCL or an
in-process loopback) or the CPU oracle (prefix "orc_", host buffers, gloo);
the driver itself holds no arithmetic of the path.
"""
from __future__ import annotations

import ctypes as C

import torch


def _check(lib, prefix, rc, what):
    if rc is not None and rc < 0:
        msg = getattr(lib, prefix + "last_error")()
        raise RuntimeError(f"{prefix}{what} failed ({rc}): {msg.decode() if msg else ''}")
    return rc


class Tile:
    """Buffers of one strip: merit partials, gathered partials, 2x2 halo and
    2x2 birth-record buffers (index 0 = the tile above, 1 = the tile below)."""

    def __init__(self, lib, prefix, handle, row0, ntiles, device, arena_bytes=0):
        self.lib, self.p, self.h = lib, prefix, handle
        self.row0 = row0
        self.ntiles = ntiles
        _check(lib, prefix, getattr(lib, prefix + "set_tile")(handle, row0, arena_bytes), "set_tile")
        pb, hb, rb = C.c_int64(), C.c_int64(), C.c_int64()
        _check(lib, prefix, getattr(lib, prefix + "tile_buffer_bytes")(
            handle, C.byref(pb), C.byref(hb), C.byref(rb)), "tile_buffer_bytes")
        self.n_part = pb.value // 8
        u8 = dict(dtype=torch.uint8, device=device)
        self.part = torch.zeros(self.n_part, dtype=torch.float64, device=device)
        self.gathered = torch.zeros(self.n_part * ntiles, dtype=torch.float64, device=device)
        self.halo_send = [torch.zeros(hb.value, **u8) for _ in range(2)]
        self.halo_recv = [torch.zeros(hb.value, **u8) for _ in range(2)]
        self.rec_send = [torch.zeros(rb.value, **u8) for _ in range(2)]
        self.rec_recv = [torch.zeros(rb.value, **u8) for _ in range(2)]
        ptrs = [C.c_void_p(t.data_ptr()) for t in
                self.halo_send + self.halo_recv + self.rec_send + self.rec_recv]
        _check(lib, prefix, getattr(lib, prefix + "set_tile_buffers")(handle, *ptrs),
               "set_tile_buffers")
        self.resources_changed(device)

    def resources_changed(self, device):
        """(Re)size the resource edge-row buffers after avgpu_load_resources."""
        lib, prefix, handle = self.lib, self.p, self.h
        sb = C.c_int64()
        _check(lib, prefix, getattr(lib, prefix + "tile_res_bytes")(handle, C.byref(sb)), "tile_res_bytes")
        f64 = dict(dtype=torch.float64, device=device)
        self.res_send = [torch.zeros(max(1, sb.value // 8), **f64) for _ in range(2)]
        self.res_recv = [torch.zeros(max(1, sb.value // 8), **f64) for _ in range(2)]
        self.has_res_rows = sb.value > 0
        ptrs = [C.c_void_p(t.data_ptr()) for t in self.res_send + self.res_recv]
        _check(lib, prefix, getattr(lib, prefix + "set_tile_res_buffers")(handle, *ptrs),
               "set_tile_res_buffers")
        self.cons = torch.zeros(16, dtype=torch.int64, device=device)   # AVGPU_MAX_RESOURCES

    def call(self, name, *args):
        return _check(self.lib, self.p, getattr(self.lib, self.p + name)(self.h, *args), name)


def _buffers(kind):
    return {"halo": ("halo_send", "halo_recv"), "records": ("rec_send", "rec_recv"),
            "resources": ("res_send", "res_recv")}[kind]


class LoopbackTransport:
    """All strips in this process (tests on one GPU, or the CPU oracle):
    exchanges are tensor copies in tile order on the current stream."""

    def all_gather(self, tiles):
        full = torch.cat([t.part for t in tiles])
        for t in tiles:
            t.gathered.copy_(full)

    def exchange_start(self, tiles, kind):
        self.exchange(tiles, kind)

    def exchange_wait(self, pending):
        pass

    def exchange(self, tiles, kind):
        T = len(tiles)
        for i, t in enumerate(tiles):
            up, down = tiles[(i - 1) % T], tiles[(i + 1) % T]
            send, recv = _buffers(kind)
            getattr(t, recv)[0].copy_(getattr(up, send)[1])
            getattr(t, recv)[1].copy_(getattr(down, send)[0])

    def all_reduce_sum(self, tiles):
        total = sum(t.cons for t in tiles)
        for t in tiles:
            t.cons.copy_(total)


class DistTransport:
    """One strip per rank over torch.distributed (backend "nccl" = RCCL over
    xGMI on MI355X, or "gloo" for the CPU oracle).  Strip k belongs to rank k;
    the tile above rank r is rank r-1 (mod T), the tile below rank r+1."""

    def __init__(self, dist, group=None):
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def all_gather(self, tiles):
        (t,) = tiles
        if hasattr(self.dist, "all_gather_into_tensor") and t.part.is_cuda:
            self.dist.all_gather_into_tensor(t.gathered, t.part, group=self.group)
        else:
            chunks = list(t.gathered.split(t.n_part))
            self.dist.all_gather(chunks, t.part, group=self.group)

    def all_reduce_sum(self, tiles):
        (t,) = tiles
        self.dist.all_reduce(t.cons, group=self.group)   # int64 sum == the uint64 sum mod 2^64

    def exchange(self, tiles, kind):
        self.exchange_wait(self.exchange_start(tiles, kind))

    def exchange_wait(self, pending):
        for w in pending:
            w.wait()

    def exchange_start(self, tiles, kind):
        """issue the neighbour exchange; the returned works are waited by
        exchange_wait (on "nccl": kernels launched in between run beside it)"""
        (t,) = tiles
        send, recv = (getattr(t, n) for n in _buffers(kind))
        up = (self.rank - 1) % self.world
        down = (self.rank + 1) % self.world
        d = self.dist
        # sends [to above, to below], receives [from below, from above]: with
        # two strips both peers are the same rank, and point-to-point messages
        # between a pair match in issue order, so this order pairs each send
        # with the receive of the same edge.
        ops = [d.P2POp(d.isend, send[0], up, self.group), d.P2POp(d.isend, send[1], down, self.group),
               d.P2POp(d.irecv, recv[1], down, self.group), d.P2POp(d.irecv, recv[0], up, self.group)]
        return d.batch_isend_irecv(ops)


class StagedTransport(DistTransport):
    """DistTransport over a host-only backend ("gloo") for device strips:
    every collective step copies the device buffers to host tensors (the copy
    waits for the strip's stream, on which the product library runs),
    exchanges them, and copies the result back before the next launch.  This
    is how two ranks that share ONE GPU -- which RCCL refuses -- run the
    product's strips across processes (tests/test_tiles_mp_gpu.py); on a node
    with a GPU per rank, DistTransport over "nccl" keeps everything on the
    device."""

    def all_gather(self, tiles):
        (t,) = tiles
        host = t.part.cpu()
        out = [torch.empty_like(host) for _ in range(self.world)]
        self.dist.all_gather(out, host, group=self.group)
        t.gathered.copy_(torch.cat(out))

    def all_reduce_sum(self, tiles):
        (t,) = tiles
        host = t.cons.cpu()
        self.dist.all_reduce(host, group=self.group)
        t.cons.copy_(host)

    def exchange_start(self, tiles, kind):
        (t,) = tiles
        send, recv = (getattr(t, n) for n in _buffers(kind))
        hs = [b.cpu() for b in send]
        hr = [torch.empty_like(hs[0]) for _ in range(2)]
        up = (self.rank - 1) % self.world
        down = (self.rank + 1) % self.world
        d = self.dist
        ops = [d.P2POp(d.isend, hs[0], up, self.group), d.P2POp(d.isend, hs[1], down, self.group),
               d.P2POp(d.irecv, hr[1], down, self.group), d.P2POp(d.irecv, hr[0], up, self.group)]
        return d.batch_isend_irecv(ops), hs, hr, recv

    def exchange_wait(self, pending):
        works, _, hr, recv = pending
        for w in works:
            w.wait()
        for k in range(2):
            recv[k].copy_(hr[k])


class StripWorld:
    """Runs updates of the strips this process holds (`tiles`, in global row
    order) with `transport` doing the collective steps."""

    def __init__(self, tiles, transport):
        self.tiles = tiles
        self.tr = transport

    def update(self):
        tiles = self.tiles
        for t in tiles:
            t.call("tile_partials", C.c_void_p(t.part.data_ptr()))
        self.tr.all_gather(tiles)
        # the update's batch steps: the same K on every strip (the gathered
        # predictors are the same bytes everywhere)
        k = C.c_int(1)
        tiles[0].call("tile_steps", C.c_void_p(tiles[0].gathered.data_ptr()), tiles[0].ntiles, C.byref(k))
        self.steps = k.value
        for sub in range(k.value):
            if sub > 0:
                for t in tiles:
                    t.call("tile_partials", C.c_void_p(t.part.data_ptr()))
                self.tr.all_gather(tiles)
            self._step(sub, k.value)

    def _step(self, sub, nsteps):
        tiles = self.tiles
        if tiles[0].has_res_rows and sub == 0:    # the spatial step runs at step 0
            self.tr.exchange(tiles, "resources")
        for t in tiles:
            t.call("tile_begin_step", C.c_void_p(t.gathered.data_ptr()), t.ntiles, sub, nsteps)
        self.tr.exchange(tiles, "halo")
        # round 0: the picks and their kill times, then (with the neighbours'
        # kill times on the edge rows) the cancellations and round 0's
        # claims; then one launch and one exchange per placement round: round
        # r's launch resolves round r - 1 with the claims both strips sent and
        # picks round r; the claims on both sides of each strip edge go out
        # together
        for rnd, phase in ((0, 0), (0, 3), (1, 0), (2, 0), (3, 0)):
            for t in tiles:
                t.call("tile_place", rnd, phase)
            self.tr.exchange(tiles, "halo")
        for t in tiles:
            t.call("tile_place", 3, 1)     # round 3 resolved, the halo offspring packed
        pending = self.tr.exchange_start(tiles, "records")
        for t in tiles:
            t.call("tile_place", 3, 2)     # this strip's own winners, beside the exchange
        self.tr.exchange_wait(pending)
        for t in tiles:
            t.call("tile_finish", None)
        pools = [t.call("tile_res_cons", C.c_void_p(t.cons.data_ptr())) for t in tiles]
        if pools[0] > 0:
            self.tr.all_reduce_sum(tiles)
            for t in tiles:
                t.call("tile_res_settle", C.c_void_p(t.cons.data_ptr()))
