"""Readers for the reference's file formats on this path.

Host-side mirror of the reference's config plumbing, limited to what the
heads-CPU hot path consumes:

* ``avida.cfg``            -- cAvidaConfig / cInitFile (main/cAvidaConfig.h:71-135,
                              tools/cInitFile.cc:145-200, ``#include`` supported)
* instruction sets         -- new ``INSTSET``/``INST`` format and the legacy
                              ``name redundancy`` format (cpu/cHardwareManager.cc:59-237,
                              cpu/cInstSet.cc:152-312)
* ``environment.cfg``      -- REACTION lines (main/cEnvironment.cc:1185-1211)
* ``events.cfg``           -- ``u begin Inject`` / ``LoadPopulation`` / ``Exit``
                              (main/cEventList.cc:387-420)
* ``.org`` genomes, ``.pop`` genotype files and ``.spop`` structured population
  files (util/GenomeLoader.cc:34-104, main/cPopulation.cc:6294-7000)

Paths are relative to avida-core/source/ of the reference.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field

# handler ids == include/avida_gpu.h enum avgpu_handler
HANDLER_NAMES = [
    "nop-A", "nop-B", "nop-C", "if-n-equ", "if-less", "pop", "push", "swap-stk",
    "swap", "shift-r", "shift-l", "inc", "dec", "add", "sub", "nand", "IO",
    "h-alloc", "h-divide", "h-copy", "h-search", "mov-head", "jmp-head",
    "get-head", "if-label", "set-flow",
]
HANDLER_ID = {n: i for i, n in enumerate(HANDLER_NAMES)}

TASK_NAMES = ["not", "nand", "and", "orn", "or", "andn", "nor", "xor", "equ"]
TASK_ID = {n: i for i, n in enumerate(TASK_NAMES)}
PROC_TYPES = {"add": 0, "mult": 1, "pow": 2}
INT32_MAX = 2**31 - 1


@dataclass
class InstSet:
    """cInstSet: op code i (INST line order) -> handler, redundancy (mutation weight)."""
    name: str
    names: list
    redundancy: list

    @property
    def handlers(self):
        return [HANDLER_ID[n] for n in self.names]

    def symbol(self, op: int) -> str:
        # Instruction::GetSymbol: a..z then A..Z (include/public/avida/core/InstructionSequence.h)
        return chr(ord("a") + op) if op < 26 else chr(ord("A") + op - 26)

    def op_of_symbol(self, ch: str) -> int:
        if "a" <= ch <= "z":
            return ord(ch) - ord("a")
        if "A" <= ch <= "Z":
            return ord(ch) - ord("A") + 26
        raise ValueError(f"bad genome symbol {ch!r}")

    def parse_sequence(self, s: str) -> bytes:
        return bytes(self.op_of_symbol(c) for c in s.strip())

    def to_sequence(self, ops) -> str:
        return "".join(self.symbol(o) for o in ops)

    def op_of_name(self, name: str) -> int:
        return self.names.index(name)


def _strip(line: str) -> str:
    return line.split("#", 1)[0].strip()


def read_instset_lines(lines, legacy=None) -> InstSet:
    """Parse an instruction set from config lines (new or legacy format)."""
    names, red = [], []
    setname = "heads_default"
    for raw in lines:
        line = _strip(raw)
        if not line:
            continue
        toks = line.split()
        if toks[0] == "INSTSET":
            setname = toks[1].split(":")[0]
            continue
        if toks[0] == "INST":
            spec = toks[1].split(":")
            nm, r = spec[0], 1
            for kv in spec[1:]:
                k, _, v = kv.partition("=")
                if k == "redundancy":
                    r = int(float(v))  # int-truncated (cpu/cInstSet.cc:231)
            names.append(nm)
            red.append(r)
            continue
        if legacy is False:
            continue
        # legacy: "name redundancy [cost ...]" (cpu/cHardwareManager.cc:184-237)
        if toks[0] in HANDLER_ID:
            names.append(toks[0])
            red.append(int(float(toks[1])) if len(toks) > 1 else 1)
    for n in names:
        if n not in HANDLER_ID:
            raise ValueError(f"instruction {n!r} is outside the heads_default hot path")
    return InstSet(setname, names, red)


def read_instset(path: str) -> InstSet:
    with open(path) as f:
        return read_instset_lines(f.readlines())


@dataclass
class Reaction:
    name: str
    task: int
    proc_type: int = 0           # cReactionProcess default PROCTYPE_ADD (main/cReactionProcess.h:73-88)
    value: float = 1.0
    max_number: float = 1.0
    min_count: int = 0
    max_count: int = INT32_MAX
    has_requisite: int = 0
    resource: int = 0            # 1 + resource index, 0 = infinite
    min_number: float = 0.0
    max_fraction: float = 1.0
    depletable: int = 1


RES_NONE = -99                   # cResource::NONE


@dataclass
class Resource:
    """RESOURCE name:... (main/cEnvironment.cc:474-661; defaults main/cResource.cc:44-64)"""
    name: str
    geometry: int = 0            # 0 global, 1 grid, 2 torus
    initial: float = 0.0
    inflow: float = 0.0
    outflow: float = 0.0
    inflow_x1: int = RES_NONE
    inflow_x2: int = RES_NONE
    inflow_y1: int = RES_NONE
    inflow_y2: int = RES_NONE
    outflow_x1: int = RES_NONE
    outflow_x2: int = RES_NONE
    outflow_y1: int = RES_NONE
    outflow_y2: int = RES_NONE
    xdiffuse: float = 1.0
    ydiffuse: float = 1.0
    xgravity: float = 0.0
    ygravity: float = 0.0


@dataclass
class CellResource:
    resource: int
    cell: int
    initial: float = 0.0
    inflow: float = 0.0
    outflow: float = 0.0


class Environment(list):
    """The REACTION list (what avgpu_load_env takes) plus .resources / .cells."""
    def __init__(self):
        super().__init__()
        self.resources = []
        self.cells = []


def _cell_list(spec):
    """cStringUtil::ReturnArray: comma separated ids and a..b ranges"""
    out = []
    for part in spec.split(","):
        if ".." in part:
            a, b = part.split("..")
            out.extend(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


def _parse_resource(tok, env, geometry_names={"global": 0, "grid": 1, "torus": 2}):
    name, _, rest = tok.partition(":")
    res = next((r for r in env.resources if r.name == name), None)
    if res is None:
        res = Resource(name)
        env.resources.append(res)
    keys = {"inflowx": "inflow_x1", "inflowx1": "inflow_x1", "inflowx2": "inflow_x2",
            "inflowy": "inflow_y1", "inflowy1": "inflow_y1", "inflowy2": "inflow_y2",
            "outflowx": "outflow_x1", "outflowx1": "outflow_x1", "outflowx2": "outflow_x2",
            "outflowy": "outflow_y1", "outflowy1": "outflow_y1", "outflowy2": "outflow_y2"}
    for kv in rest.split(":"):
        if not kv:
            continue
        k, _, v = kv.partition("=")
        k = k.lower()
        if k in ("inflow", "outflow", "initial", "xdiffuse", "ydiffuse", "xgravity", "ygravity"):
            setattr(res, k, float(v))
        elif k == "geometry":
            if v.lower() not in geometry_names:
                raise ValueError(f"resource geometry {v!r} not supported on this path")
            res.geometry = geometry_names[v.lower()]
        elif k in keys:
            setattr(res, keys[k], int(v))
        else:
            raise ValueError(f"resource setting {k!r} not supported on this path")
    # one-point boxes (main/cEnvironment.cc:636-657)
    if res.inflow_x1 >= 0 and res.inflow_x2 == RES_NONE:
        res.inflow_x2 = res.inflow_x1
    if res.inflow_y1 >= 0 and res.inflow_y2 == RES_NONE:
        res.inflow_y2 = res.inflow_y1
    if res.outflow_x1 > 0 and res.outflow_x2 == RES_NONE:
        res.outflow_x2 = res.outflow_x1
    if res.outflow_y1 > 0 and res.outflow_y2 == RES_NONE:
        res.outflow_y2 = res.outflow_y1


def _parse_cell(tok, env):
    """CELL name:cells[:initial=..:inflow=..:outflow=..] (main/cEnvironment.cc:663-755)"""
    parts = tok.split(":")
    name, cells = parts[0], _cell_list(parts[1])
    idx = next((i for i, r in enumerate(env.resources) if r.name == name), None)
    if idx is None:
        env.resources.append(Resource(name, geometry=1, xdiffuse=0.0, ydiffuse=0.0))
        idx = len(env.resources) - 1
    vals = {"initial": 0.0, "inflow": 0.0, "outflow": 0.0}
    for kv in parts[2:]:
        k, _, v = kv.partition("=")
        if k not in vals:
            raise ValueError(f"CELL setting {k!r} unknown")
        vals[k] = float(v)
    for c in cells:
        old = next((x for x in env.cells if x.resource == idx and x.cell == c), None)
        if old:
            old.initial, old.inflow, old.outflow = vals["initial"], vals["inflow"], vals["outflow"]
        else:
            env.cells.append(CellResource(idx, c, **vals))


def read_environment(path: str):
    """REACTION name task process:... requisite:... (main/cEnvironment.cc:1185-1211),
    RESOURCE and CELL lines (:474-755).  Returns an Environment (a list of
    Reaction with .resources and .cells)."""
    with open(path) as f:
        return parse_environment(f.read())


def parse_environment(text: str):
    """read_environment on the text of an environment file"""
    out = Environment()
    text = re.sub(r"\\[ \t]*\r?\n[ \t]*", "", text)   # "\" joins the next line
    for raw in text.splitlines():
            line = _strip(raw)
            if not line:
                continue
            toks = line.split()
            if toks[0] == "RESOURCE":
                for tok in toks[1:]:
                    _parse_resource(tok, out)
                continue
            if toks[0] == "CELL":
                for tok in toks[1:]:
                    _parse_cell(tok, out)
                continue
            if toks[0] != "REACTION":
                raise ValueError(f"environment keyword {toks[0]} not supported on this path")
            name, task = toks[1], toks[2].split(":")[0]
            if task not in TASK_ID:
                raise ValueError(f"task {task!r} is not a logic-9 task")
            r = Reaction(name, TASK_ID[task])
            for tok in toks[3:]:
                kind, _, rest = tok.partition(":")
                kv = dict(p.split("=", 1) for p in rest.split(":") if "=" in p)
                if kind == "process":
                    if "type" in kv:
                        r.proc_type = PROC_TYPES[kv["type"]]
                    if "value" in kv:
                        r.value = float(kv["value"])
                    if "max" in kv:
                        r.max_number = float(kv["max"])
                    if "min" in kv:
                        r.min_number = float(kv["min"])
                    if "frac" in kv:
                        r.max_fraction = min(1.0, float(kv["frac"]))
                    if "depletable" in kv:
                        r.depletable = int(kv["depletable"])
                    if "resource" in kv and kv["resource"] not in ("none", ""):
                        names = [x.name for x in out.resources]
                        if kv["resource"] not in names:
                            raise ValueError(f"unknown resource {kv['resource']!r}")
                        r.resource = 1 + names.index(kv["resource"])
                    for k in kv:
                        if k not in ("type", "value", "max", "min", "frac", "depletable", "resource"):
                            raise ValueError(f"process setting {k!r} not supported on this path")
                elif kind == "requisite":
                    r.has_requisite = 1
                    if "max_count" in kv:
                        r.max_count = int(kv["max_count"])
                    if "min_count" in kv:
                        r.min_count = int(kv["min_count"])
            out.append(r)
    return out


def _read_cfg_lines(path, seen=None):
    seen = seen or set()
    base = os.path.dirname(path)
    lines = []
    with open(path) as f:
        for raw in f:
            s = raw.strip()
            if s.startswith("#include"):
                inc = s[len("#include"):].strip()
                if "=" in inc:
                    inc = inc.split("=", 1)[1]
                p = os.path.join(base, inc)
                if p not in seen and os.path.exists(p):
                    seen.add(p)
                    lines.extend(_read_cfg_lines(p, seen))
                continue
            lines.append(raw)
    return lines


@dataclass
class AvidaConfig:
    values: dict = field(default_factory=dict)
    instset: InstSet | None = None

    def get(self, key, default=None):
        return self.values.get(key, default)


CFG_KEYS_INT = {
    "WORLD_X": 60, "WORLD_Y": 60, "WORLD_GEOMETRY": 2, "AVE_TIME_SLICE": 30,
    "SLICING_METHOD": 1, "BASE_MERIT_METHOD": 4, "BASE_CONST_MERIT": 100,
    "REQUIRE_ALLOCATE": 1, "DEATH_METHOD": 2, "AGE_LIMIT": 20, "ALLOC_METHOD": 0,
    "DIVIDE_METHOD": 1, "MAX_LABEL_EXE_SIZE": 1, "BIRTH_METHOD": 0, "PREFER_EMPTY": 1,
    "ALLOW_PARENT": 1, "TEST_CPU_TIME_MOD": 20, "MIN_GENOME_SIZE": 0,
    "MAX_GENOME_SIZE": 0, "INHERIT_MERIT": 1, "RANDOM_SEED": -1,
    "INST_SET_LOAD_LEGACY": 0, "SLIP_FILL_MODE": 0,
}
CFG_KEYS_FLOAT = {
    "DEFAULT_BONUS": 1.0, "COPY_MUT_PROB": 0.0075, "COPY_INS_PROB": 0.0,
    "COPY_DEL_PROB": 0.0, "DIVIDE_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.05,
    "DIVIDE_DEL_PROB": 0.05, "OFFSPRING_SIZE_RANGE": 2.0, "MIN_COPIED_LINES": 0.5,
    "MIN_EXE_LINES": 0.5, "MERIT_DEFAULT_BONUS": 0.0, "REQUIRED_BONUS": 0.0,
    "DIVIDE_SLIP_PROB": 0.0, "DIVIDE_UNIFORM_PROB": 0.0,
}


def read_avida_cfg(path: str | None = None, overrides: dict | None = None) -> AvidaConfig:
    """cAvidaConfig::Load; unknown keys are kept verbatim, ``-set`` style overrides win."""
    vals = dict(CFG_KEYS_INT)
    vals.update(CFG_KEYS_FLOAT)
    inst_lines = []
    if path:
        for raw in _read_cfg_lines(path):
            line = _strip(raw)
            if not line:
                continue
            toks = line.split()
            if toks[0] in ("INSTSET", "INST"):
                inst_lines.append(line)
                continue
            key = toks[0]
            val = toks[1] if len(toks) > 1 else ""
            if key in CFG_KEYS_INT:
                vals[key] = int(float(val))
            elif key in CFG_KEYS_FLOAT:
                vals[key] = float(val)
            else:
                vals[key] = val
    for k, v in (overrides or {}).items():
        vals[k] = v
    cfg = AvidaConfig(vals)
    if inst_lines:
        cfg.instset = read_instset_lines(inst_lines, legacy=False)
    return cfg


def read_org(path: str, instset: InstSet) -> bytes:
    """.org file: one instruction name per line (util/GenomeLoader.cc:34-104)."""
    ops = []
    with open(path) as f:
        for raw in f:
            line = _strip(raw)
            if line:
                ops.append(instset.op_of_name(line.split()[0]))
    return bytes(ops)


@dataclass
class Genotype:
    id: int
    num_cpus: int
    length: int
    merit: float
    gest_time: int
    fitness: float
    sequence: str
    cells: list | None = None        # .spop "cells" (structured population)
    gest_offset: list | None = None  # .spop "gest_offset" (CPU cycles into the gestation)
    props: dict = field(default_factory=dict)


def _int_list(v):
    return [int(x) for x in v.split(",")] if v not in (None, "", "(none)") else None


def read_pop(path: str):
    """.pop / .spop genotype_data file (#format line names the columns;
    cPopulation::LoadPopulation reads num_units, falling back to num_cpus,
    main/cPopulation.cc:6747-6766)."""
    fmt = None
    out = []
    with open(path) as f:
        for raw in f:
            if raw.startswith("#format"):
                fmt = raw.split()[1:]
                continue
            if raw.startswith("#") or not raw.strip():
                continue
            toks = raw.split()
            rec = dict(zip(fmt, toks))
            num = rec.get("num_units", rec.get("num_cpus", 1))
            out.append(Genotype(
                int(rec.get("id", 0)), int(num),
                int(rec.get("length", len(rec["sequence"]))),
                float(rec.get("merit", 0)), int(float(rec.get("gest_time", 0))),
                float(rec.get("fitness", 0)), rec["sequence"],
                _int_list(rec.get("cells")), _int_list(rec.get("gest_offset")), rec))
    return out


def read_events(path: str):
    """events.cfg subset: returns list of (trigger, start, action, args)."""
    ev = []
    with open(path) as f:
        for raw in f:
            line = _strip(raw)
            if not line:
                continue
            toks = line.split()
            ev.append((toks[0], toks[1], toks[2], toks[3:]))
    return ev


def parse_detail_dat(path: str):
    """analyze DETAIL output: returns (format_names, rows)."""
    fmt, rows = None, []
    with open(path) as f:
        for raw in f:
            if raw.startswith("#format"):
                fmt = raw.split()[1:]
                continue
            if raw.startswith("#") or not raw.strip():
                continue
            rows.append(raw.split())
    return fmt, rows
