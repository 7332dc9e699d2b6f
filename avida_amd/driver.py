"""Avida2Driver restated over the C-ABI (targets/avida/Avida2Driver.cc:91-163).

Reads a reference config directory (avida.cfg, the instruction set, the
environment file with REACTION / RESOURCE / CELL lines, events.cfg), runs the
world on the MI355X path (`libavida_gpu.so`) and writes the reference's data
files (avida_amd/datafiles.py).  The update loop keeps the reference's event
timing: "begin" events run before update 0; an event of update u runs after
update u has been processed (the next iteration's GetEvents), so a print at u
shows the state at the end of update u, and "u N Exit" ends after update N.

Events on this path (main/cEventList.cc syntax "u <start>[:<interval>[:<end>]]"):
Inject <org> [cell] [merit], InjectAll <org> [merit], InjectSequence <seq>
[start] [end] [merit], LoadPopulation <file> [update] [cellid_offset] (.pop /
.spop, avida_amd/population.py), SavePopulation [name] (<name>-<update>.spop),
Print{Count,Average,Tasks,Time,Resource,Dominant}Data [file], SaveCheckpoint
[file] / LoadCheckpoint <file> (full hardware state, avida_amd/checkpoint.py),
Exit.  Other Print* events write nothing; anything else is an error.

    python -m avida_amd.driver -c <config dir> -d <data dir> [-u MAX_UPDATES]
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys

from . import capi, checkpoint, datafiles, files, population, systematics


class ProductWorld:
    """The world on the GPU through libavida_gpu.so (same methods as the
    tests' oracle Backend, so the driver runs on either)."""

    def __init__(self, cfg, iset, env, ncells=0, device=0, serial=False):
        self.lib, self.p = capi.load_product(), "avgpu_"
        # serial=True: every update under the reference's own schedule
        # (avgpu_run_serial_updates: per-step merit-weighted picks, births at
        # once) instead of the batch update
        self.serial = serial
        self.h = self.lib.avgpu_create(C.byref(cfg), device, ncells)
        if not self.h:
            raise RuntimeError(self.lib.avgpu_last_error().decode())
        self.cfg = cfg
        self.ncells = ncells or cfg.world_x * cfg.world_y
        hid = (C.c_uint8 * len(iset.names))(*iset.handlers)
        red = (C.c_int32 * len(iset.names))(*iset.redundancy)
        self._call("load_instset", self.h, len(iset.names), hid, red)
        self.nres = len(getattr(env, "resources", []))
        if self.nres:
            ra, ca = capi.resources_arrays(env.resources, env.cells)
            self._call("load_resources", self.h, self.nres, ra, len(env.cells), ca)
        self._call("load_env", self.h, len(env), capi.reactions_array(env))

    def _call(self, name, *args):
        rc = getattr(self.lib, self.p + name)(*args)
        if rc is not None and rc < 0:
            raise RuntimeError(f"{self.p}{name}: {self.lib.avgpu_last_error().decode()}")
        return rc

    def set_orgs(self, first, genomes, merits=None, deterministic=False):
        n = len(genomes)
        blob = b"".join(genomes)
        buf = (C.c_uint8 * max(1, len(blob))).from_buffer_copy(blob or b"\0")
        lens = (C.c_int32 * n)(*[len(g) for g in genomes])
        m = (C.c_double * n)(*(merits or [0.0] * n))
        self._call("set_orgs", self.h, first, n, buf, lens, m, None, 1 if deterministic else 0)

    def run_update(self):
        st = capi.AvgpuUpdateStats()
        if self.serial:
            self._call("run_serial_updates", self.h, 1, C.byref(st))
        else:
            self._call("run_update", self.h, C.byref(st))
        return st

    def kill(self, cell):
        self._call("kill", self.h, cell)

    def states(self, first, count, cap=capi.MAX_GENOME):
        st = (capi.AvgpuCpuState * count)()
        ops = (C.c_uint8 * (count * cap))()
        fl = (C.c_uint8 * (count * cap))()
        self._call("get_states", self.h, first, count, st, ops, fl, cap)
        return st, bytes(ops), bytes(fl)

    def test_genomes(self, genomes, flags_cap=2049):
        n = len(genomes)
        blob = b"".join(genomes)
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        lens = (C.c_int32 * n)(*[len(g) for g in genomes])
        res = (capi.AvgpuTestResult * n)()
        flags = C.create_string_buffer(n * flags_cap)
        self._call("test_genomes", self.h, n, buf, lens, res, flags, flags_cap, None)
        return [(res[i], None, None) for i in range(n)]

    def census(self, first=0, count=None):
        return capi.get_census(self.lib, self.p, self.h, first, self.ncells - first if count is None else count)

    def resources(self, spatial=False):
        lv = (C.c_double * max(1, self.nres))()
        self._call("get_resources", self.h, lv, None)
        return list(lv[:self.nres]), None

    def checkpoint(self, path):
        checkpoint.save(self.lib, self.p, self.h, self.ncells, self.nres, path)

    def restore(self, path):
        return checkpoint.load(self.lib, self.p, self.h, path)

    def close(self):
        if self.h:
            self.lib.avgpu_destroy(self.h)
            self.h = None


def load_config(config_dir):
    """(avida config, instruction set, environment, events) of a reference config dir"""
    cfg = files.read_avida_cfg(os.path.join(config_dir, "avida.cfg"))
    iset = cfg.instset
    if iset is None:
        name = cfg.get("INST_SET", "-")
        path = os.path.join(config_dir, name if name not in ("-", "") else "instset-heads.cfg")
        iset = files.read_instset(path)
    env = files.read_environment(os.path.join(config_dir, cfg.get("ENVIRONMENT_FILE", "environment.cfg")))
    events = files.read_events(os.path.join(config_dir, cfg.get("EVENT_FILE", "events.cfg")))
    return cfg, iset, env, events


def _fires(trigger, start, u):
    """does an update event "u <start>[:<interval>[:<end>]]" fire after update u?"""
    if trigger != "u":
        raise ValueError(f"event trigger {trigger!r} is not supported on this path")
    parts = start.split(":")
    if parts[0] == "begin":
        return False
    s = int(parts[0])
    if len(parts) == 1:
        return u == s
    step = int(parts[1])
    end = parts[2] if len(parts) > 2 else "end"
    if u < s or (end != "end" and u > int(end)):
        return False
    return (u - s) % step == 0


class Driver:
    def __init__(self, config_dir, data_dir, make_world=None, seed=None):
        self.config_dir = config_dir
        acfg, self.iset, self.env, self.events = load_config(config_dir)
        self.cfg = capi.cfg_from_avida(acfg, seed=seed)
        self.world = (make_world or ProductWorld)(self.cfg, self.iset, self.env)
        self.rec = datafiles.StatsRecorder(data_dir, [r.name for r in getattr(self.env, "resources", [])])
        self.data_dir = data_dir
        # genotype classification runs every update when a data file needs it
        # (the reference's systematics manager classifies every birth)
        need = {"PrintCountData", "PrintDominantData", "SavePopulation", "PrintAverageData"}
        self.arbiter = systematics.GenotypeArbiter(int(acfg.get("THRESHOLD", 3))) \
            if any(e[2] in need for e in self.events) else None
        self.rec.arbiter = self.arbiter
        self.done = False
        self.update = -1

    def _org(self, name):
        return files.read_org(os.path.join(self.config_dir, name), self.iset)

    def _action(self, action, args):
        w = self.world
        if action == "Inject":
            cell = int(args[1]) if len(args) > 1 else 0
            merit = float(args[2]) if len(args) > 2 else -1.0
            w.set_orgs(cell, [self._org(args[0])], [max(0.0, merit)], deterministic=False)
            self.rec.injected += 1
        elif action == "InjectAll":
            g = self._org(args[0])
            merit = float(args[1]) if len(args) > 1 else -1.0
            n = self.cfg.world_x * self.cfg.world_y
            w.set_orgs(0, [g] * n, [max(0.0, merit)] * n, deterministic=False)
            self.rec.injected += n
        elif action.lower() == "injectsequence":
            g = self.iset.parse_sequence(args[0])
            start = int(args[1]) if len(args) > 1 else 0
            end = int(args[2]) if len(args) > 2 else start + 1
            merit = float(args[3]) if len(args) > 3 else -1.0
            w.set_orgs(start, [g] * (end - start), [max(0.0, merit)] * (end - start), deterministic=False)
            self.rec.injected += end - start
        if action in ("Inject", "InjectAll") or action.lower() == "injectsequence":
            if self.arbiter is not None:      # injected units are classified at once
                self.arbiter.update(w.census(), max(self.update, 0))
            return
        if action == "PrintCountData":
            self.rec.print_count(*args[:1])
        elif action == "PrintDominantData":
            self.rec.print_dominant(*args[:1])
        elif action == "PrintAverageData":
            self.rec.print_average(*args[:1])
        elif action == "PrintTasksData":
            self.rec.print_tasks(*args[:1])
        elif action == "PrintTimeData":
            self.rec.print_time(*args[:1])
        elif action == "PrintResourceData":
            self.rec.print_resource(w.resources()[0], *args[:1])
        elif action == "SavePopulation":          # actions/SaveLoadActions.cc:168-176
            name = args[0] if args else "detail"
            population.save_population(w, self.iset, self.arbiter,
                                       os.path.join(self.data_dir, f"{name}-{max(self.update, 0)}.spop"),
                                       max(self.update, 0))
        elif action == "LoadPopulation":          # actions/SaveLoadActions.cc:62-88
            if len(args) > 1 and int(args[1]) >= 0:
                self.update = int(args[1]) - 1     # SetCurrentUpdate: the next update is that one
            offset = int(args[2]) if len(args) > 2 else 0
            self.rec.injected += population.load_population(
                w, self.iset, os.path.join(self.config_dir, args[0]), w.ncells, offset)
            if self.arbiter is not None:
                self.arbiter.update(w.census(), max(self.update, 0))
        elif action == "SaveCheckpoint":
            name = args[0] if args else f"checkpoint-{self.update}.npz"
            w.checkpoint(os.path.join(self.data_dir, name))
        elif action == "LoadCheckpoint":
            self.rec.end_update(w.restore(os.path.join(self.config_dir, args[0])))
        elif action == "Exit":
            self.done = True
        elif action.startswith("Print"):
            pass   # data outside this path (genotypes, systematics ...): not written
        else:
            raise ValueError(f"event action {action!r} is not supported on this path")

    def run(self, max_updates=None):
        for trig, start, action, args in self.events:
            if start.split(":")[0] == "begin":
                self._action(action, args)
        while not self.done and (max_updates is None or self.update + 1 < max_updates):
            self.update += 1
            if self.update > 0:
                self.rec.begin_update()
            self.rec.end_update(self.world.run_update())
            if self.arbiter is not None:
                self.arbiter.update(self.world.census(), self.update)
            for trig, start, action, args in self.events:
                if _fires(trig, start, self.update):
                    self._action(action, args)
        self.rec.close()
        return self.update


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("-c", "--config", default=".")
    ap.add_argument("-d", "--data", default="data")
    ap.add_argument("-u", "--max-updates", type=int, default=None)
    ap.add_argument("-s", "--seed", type=int, default=None)
    ap.add_argument("--serial", action="store_true",
                    help="the reference's own per-step schedule (avgpu_run_serial_updates) "
                         "instead of the batch update")
    a = ap.parse_args(argv)
    mk = (lambda cfg, iset, env: ProductWorld(cfg, iset, env, serial=True)) if a.serial else None
    d = Driver(a.config, a.data, make_world=mk, seed=a.seed)
    last = d.run(a.max_updates)
    print(f"ran updates 0..{last}", file=sys.stderr)
    d.world.close()


if __name__ == "__main__":
    main()
