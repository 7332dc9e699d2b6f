"""Genotype classification on the host.

The reference files every newborn under the genotype whose instruction
sequence equals its birth genome (Systematics::GenotypeArbiter::
ClassifyNewUnit, systematics/GenotypeArbiter.cc:280-380), keeps genotypes in
abundance-ordered lists (AdjustGenotype, :423-468), names a genotype when it
reaches THRESHOLD organisms or becomes the most abundant (nameGenotype,
:482-497: "%03d-" + five base-26 letters counted per genome size) and drops it
when its last organism dies (removeGenotype, :499-530).

Here the device keys each birth genome once at activation (avgpu_census,
include/avida_gpu.h) and this class groups a world's census by key after
each update.  It is a batch restatement: births and deaths of one update are
applied together, in cell order, because the batch world itself places and
activates an update's offspring together.  Rules:

* a key not among the active genotypes becomes a new genotype; new ids are
  handed out in order of the first cell holding the key;
* a genotype whose abundance falls to 0 is removed (no lineage / passive
  references are kept -- the hot path records no parent genotype); a later
  organism with the same genome starts a new genotype, as in the reference
  once the old one left the active hash;
* threshold: abundance >= THRESHOLD, or the genotype is the most abundant
  (GenotypeArbiter.cc:320-328, :459-467); names are given in id order among
  the genotypes that cross it in one update;
* dominant (GenotypeArbiter::Begin -> getBest): the most abundant; on a tie
  the previous dominant stays (the "keep the current best" special case,
  :450-453), otherwise the lowest id.

Genotype averages (merit, gestation time, fitness, repro rate, copied size)
are the means, over the genotype's living organisms that carry a completed
gestation (gestation_time > 0: a divided parent or an offspring, which
inherits its parent's last gestation values, main/cPhenotype.cc:349-420), of
the values Genotype::HandleUnitGestation (systematics/Genotype.cc:289-301)
accumulates per gestation; the reference averages over all gestations the
genotype ever had, so the two agree while the genotype's members share their
phenotype (always for a clonal lineage), and are statistically close
otherwise.  "Executed Size of Dominant Genotype" is 0 in the reference: the
organism publishes "last_exectuted_size" (main/cOrganism.cc:67) while the
genotype reads "last_executed_size" (systematics/Genotype.cc:38, :294); it is
written as 0 here too.  With no gestation recorded the averages are 0 and max
fitness is DBL_MIN (an empty cDoubleSum, as the reference's first rows show).
"""
from __future__ import annotations

import sys

import numpy as np

GOLD = 0x9E3779B97F4A7C15
M64 = (1 << 64) - 1
DBL_MIN = sys.float_info.min


def _mix(z):
    z ^= z >> 30
    z = (z * 0xBF58476D1CE4E5B9) & M64
    z ^= z >> 27
    z = (z * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def genome_key(codes) -> int:
    """Genome key of a birth genome given as canonical instruction codes
    (the device's gk_* in avida_amd/csrc/device.h; oracle genome_key)."""
    codes = bytes(codes)
    n = len(codes)
    s = 0
    for w in range((n + 3) // 4):
        v = 0
        for j in range(4):
            if 4 * w + j < n:
                v |= (codes[4 * w + j] & 0x3F) << (8 * j)
        s = (s + _mix(((w + 1) << 32) | v)) & M64
    k = _mix(s ^ ((n * GOLD) & M64))
    return k or 1


def name_letters(num: int) -> str:
    """nameGenotype's five base-26 letters (GenotypeArbiter.cc:482-497)"""
    a = []
    for _ in range(5):
        a.append(chr(ord("a") + num % 26))
        num //= 26
    return "".join(reversed(a))


class Genotype:
    __slots__ = ("id", "key", "length", "update_born", "num_units", "total_units",
                 "threshold", "name", "cells")

    def __init__(self, gid, key, length, update_born):
        self.id, self.key, self.length, self.update_born = gid, key, length, update_born
        self.num_units = 0
        self.total_units = 0
        self.threshold = False
        self.name = "%03d-no_name" % length
        self.cells = None


class GenotypeArbiter:
    """Batch restatement of Systematics::GenotypeArbiter over census rows."""

    def __init__(self, threshold=3):
        self.threshold = threshold
        self.active = {}          # key -> Genotype
        self.next_id = 1
        self.sz_count = {}        # genome size -> names handed out
        self.tot_genotypes = 0
        self.tot_threshold = 0
        self.best = None
        self.census = None

    def _name(self, size):
        k = self.sz_count.get(size, 0)
        self.sz_count[size] = k + 1
        return "%03d-%s" % (size, name_letters(k))

    def update(self, census, update):
        """Classify one census (capi.CENSUS_DTYPE rows, one per cell)."""
        self.census = census
        alive = np.nonzero(census["genotype_key"] != 0)[0]
        keys = census["genotype_key"][alive]
        uk, first, inv, counts = np.unique(keys, return_index=True, return_inverse=True,
                                           return_counts=True)
        order = np.argsort(inv, kind="stable")
        bounds = np.concatenate([[0], np.cumsum(counts)])
        present = {}
        for j in np.argsort(first, kind="stable"):          # first-cell order
            k = int(uk[j])
            g = self.active.get(k)
            if g is None:
                c0 = alive[first[j]]
                g = Genotype(self.next_id, k, int(census["genome_length"][c0]), update)
                self.next_id += 1
                self.tot_genotypes += 1
                self.active[k] = g
            prev = g.num_units
            g.num_units = int(counts[j])
            g.total_units += max(0, g.num_units - prev)
            g.cells = alive[order[bounds[j]:bounds[j + 1]]]
            present[k] = g
        for k in [k for k in self.active if k not in present]:
            g = self.active.pop(k)
            g.num_units = 0
            if self.best is g:
                self.best = None
        if not present:
            self.best = None
            return
        top = max(g.num_units for g in present.values())
        if self.best is None or self.best.num_units != top:
            self.best = min((g for g in present.values() if g.num_units == top), key=lambda g: g.id)
        for g in sorted(present.values(), key=lambda g: g.id):
            if not g.threshold and (g.num_units >= self.threshold or g is self.best):
                g.threshold = True
                g.name = self._name(g.length)
                self.tot_threshold += 1

    # ---- cStats / data-file views ----
    def num_genotypes(self):
        return len(self.active)

    def num_threshold(self):
        return sum(1 for g in self.active.values() if g.threshold)

    def dominant(self):
        return self.best

    def genotype_averages(self, g):
        """(merit, gestation, fitness, repro rate, copied size, max fitness)
        over g's organisms with a completed gestation"""
        rows = self.census[g.cells]
        rows = rows[rows["gestation_time"] > 0]
        if len(rows) == 0:
            return 0.0, 0.0, 0.0, 0.0, 0.0, DBL_MIN
        gest = rows["gestation_time"].astype(np.float64)
        return (float(rows["merit"].mean()), float(gest.mean()), float(rows["fitness"].mean()),
                float((1.0 / gest).mean()), float(rows["copied_size"].astype(np.float64).mean()),
                float(rows["fitness"].max()))

    def dominant_row(self, update):
        """One PrintDominantData row (actions/PrintActions.cc:5405-5440), or
        None with no organisms (the reference writes nothing then)."""
        g = self.best
        if g is None:
            return None
        merit, gest, fit, repro, copied, maxfit = self.genotype_averages(g)
        # births / breed true / depth / breed in need lineage records: 0
        return [update, merit, gest, fit, repro, g.length, copied, 0.0, g.num_units,
                0, 0, 0, 0, maxfit, g.id, g.name]
