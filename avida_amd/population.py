"""Population files: cPopulation::LoadPopulation / SavePopulation restated
over the C-ABI (main/cPopulation.cc:6723-7000, :6294-6500).

LoadPopulation (.pop genotype lists and .spop structured saves):
  * every organism already in the world is killed when cellid_offset is 0
    (:6731-6732); with an offset the file's organisms join the population;
  * genotype rows are processed in DESCENDING id order (sTmpGenotype's
    operator< compares id_num with >, :6683; Apto::QSort, :6857);
  * a structured file places each organism at cells[i] + offset, otherwise
    organism k goes to cell k + offset (u_cell_id++, :6902);
  * every organism is injected (SetupInject, :6920) with the row's merit when
    it is > 0, else its test-CPU merit (GetTestMerit, :6942-6946); a
    gest_offset scales that merit by gest_time / (gest_time - offset)
    (:6948-6958), the fraction of the gestation still ahead.

SavePopulation writes the reference's structured save: one row per living
genotype (Genotype::LegacySave columns: id src src_args parents num_units
total_units length merit gest_time fitness gen_born update_born
update_deactivated depth hw_type inst_set sequence) plus cells, gest_offset
(each organism's CPU cycles into its gestation, :6330) and lineage.  Genotype
ids and averages come from the host genotype classification
(avida_amd/systematics.py); the hot path keeps no lineage, so parents are
"(none)", gen_born / depth 0 and src "div:int".  The sequence is a member's
birth genome: the device keeps only its key, so the first member whose tape
prefix still hashes to the genotype's key provides it (an organism that copied
into its own first sites cannot).
"""
from __future__ import annotations

import time

import numpy as np

from . import capi, files, systematics


def _runs(cells):
    """consecutive-cell runs of a sorted cell list: [(first, count, index0)]"""
    out = []
    i = 0
    while i < len(cells):
        j = i
        while j + 1 < len(cells) and cells[j + 1] == cells[j] + 1:
            j += 1
        out.append((cells[i], j - i + 1, i))
        i = j + 1
    return out


def load_population(world, iset: files.InstSet, path, ncells, cellid_offset=0):
    """cPopulation::LoadPopulation into `world` (driver.ProductWorld or the
    tests' oracle Backend).  Returns the number of organisms placed."""
    gts = files.read_pop(path)
    structured = any(g.cells for g in gts)
    gts.sort(key=lambda g: -g.id)
    # test-CPU merit for rows without one (one batch)
    need = [g for g in gts if not g.merit > 0]
    test_merit = {}
    if need:
        res = world.test_genomes([iset.parse_sequence(g.sequence) for g in need])
        for g, (r, _, _) in zip(need, res):
            test_merit[id(g)] = r.merit
    placed = {}                      # cell -> (genome, merit)
    u_cell = 0
    for g in gts:
        genome = iset.parse_sequence(g.sequence)
        merit0 = g.merit if g.merit > 0 else test_merit[id(g)]
        for i in range(g.num_cpus):
            cell = (g.cells[i] if structured else u_cell) + cellid_offset
            u_cell += 1
            merit = merit0
            if g.gest_offset and i < len(g.gest_offset):
                remain = float(g.gest_time) - float(g.gest_offset[i])
                if remain > 0.0 and g.gest_time > 0:
                    merit = merit * (float(g.gest_time) / remain)
            if not 0 <= cell < ncells:
                raise ValueError(f"{path}: cell {cell} outside the world")
            placed[cell] = (genome, merit)      # a later row on the same cell wins
    # KillOrganism for every organism not replaced: the world is cleared first
    # only when cellid_offset is 0 (main/cPopulation.cc:6731-6732); with an
    # offset the loaded organisms are added to the existing population
    if cellid_offset == 0:
        occ = np.nonzero(world.census()["genotype_key"] != 0)[0]
        for c in occ:
            if int(c) not in placed:
                world.kill(int(c))
    cells = sorted(placed)
    for first, count, k in _runs(cells):
        chunk = cells[k:k + count]
        world.set_orgs(first, [placed[c][0] for c in chunk], [placed[c][1] for c in chunk],
                       deterministic=False)
    return len(cells)


def save_population(world, iset: files.InstSet, arbiter, path, update, cap=capi.MAX_GENOME):
    """cPopulation::SavePopulation (structured save) of `world` after
    `update`; `arbiter` = the driver's GenotypeArbiter, updated this update."""
    census = world.census()
    if arbiter is None:
        arbiter = systematics.GenotypeArbiter()
        arbiter.update(census, update)
    handlers = iset.handlers
    inst_set = iset.name or "heads_default"
    n = len(census)
    st, ops, _ = world.states(0, n, cap)
    rows = []
    for g in sorted(arbiter.active.values(), key=lambda g: g.id):
        cells = [int(c) for c in g.cells]
        seq = None
        offsets = []
        for c in cells:
            s = st[c]
            offsets.append(s.cpu_cycles_used)
            if seq is None:
                prefix = ops[c * cap:c * cap + s.birth_length]
                if systematics.genome_key(bytes(handlers[x] for x in prefix)) == g.key:
                    seq = iset.to_sequence(prefix)
        if seq is None:          # every member copied into its own first sites
            c = cells[0]
            seq = iset.to_sequence(ops[c * cap:c * cap + st[c].birth_length])
        merit, gest, fit, _, _, _ = arbiter.genotype_averages(g)
        rows.append([g.id, "div:int", "(none)", "(none)", g.num_units, max(g.total_units, g.num_units),
                     g.length, "%g" % merit, "%g" % gest, "%g" % fit, 0, g.update_born, -1, 0, 0, inst_set,
                     seq, ",".join(map(str, cells)), ",".join(map(str, offsets)),
                     ",".join("0" for _ in cells)])
    cols = ["ID", "Source", "Source Args", "Parent ID(s)", "Number of currently living organisms",
            "Total number of organisms that ever existed", "Genome Length", "Average Merit",
            "Average Gestation Time", "Average Fitness", "Generation Born", "Update Born",
            "Update Deactivated", "Phylogenetic Depth", "Hardware Type ID", "Inst Set Name",
            "Genome Sequence", "Occupied Cell IDs", "Gestation (CPU) Cycle Offsets", "Lineage Label"]
    with open(path, "w") as f:
        f.write("#filetype genotype_data\n")
        f.write("#format id src src_args parents num_units total_units length merit gest_time fitness "
                "gen_born update_born update_deactivated depth hw_type inst_set sequence cells "
                "gest_offset lineage \n")
        f.write("# Structured Population Save\n")
        f.write("# " + time.strftime("%a %b %d %H:%M:%S %Y") + "\n")
        for i, c in enumerate(cols):
            f.write("#%3d: %s\n" % (i + 1, c))
        f.write("\n")
        for r in rows:
            f.write(" ".join(str(x) for x in r) + " \n")
    return len(rows)
