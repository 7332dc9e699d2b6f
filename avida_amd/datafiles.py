"""Reference-format data files from the per-update statistics (SURVEY.md 8f
rank 1): count.dat, average.dat, tasks.dat, time.dat, resource.dat as
cStats::Print{Count,Average,Tasks,Time,Resource}Data write them
(main/cStats.cc:1081-1105, :658-700, :1202-1224, :1675-1687, :1551-1579):
the same header comments and column legends, one row per printed update,
numbers in C++ ostream default format (6 significant digits, '%g').

dominant.dat (PrintDominantData, actions/PrintActions.cc:5405-5440) and
count.dat's genotype columns come from the host genotype classification
(avida_amd/systematics.py).  Columns the hot path does not track (species / lineage counts,
breed-true, thread counts, repro rate, copied / executed size averages,
neutral metric, lineage label) are written as 0 and listed in
UNTRACKED; the tracked ones come from avgpu_update_stats.
"""
from __future__ import annotations

import os
import time

TASK_NAMES = ["Not", "Nand", "And", "OrNot", "Or", "AndNot", "Nor", "Xor", "Equals"]

COUNT_COLS = ["update", "number of insts executed this update", "number of organisms",
              "number of different genotypes", "number of different threshold genotypes",
              "(deprecated) number of different species", "(deprecated) number of different threshold species",
              "(deprecated) number of different lineages", "number of births in this update",
              "number of deaths in this update", "number of breed true", "number of breed true organisms?",
              "number of no-birth organisms", "number of single-threaded organisms",
              "number of multi-threaded organisms", "number of modified organisms"]
AVERAGE_COLS = ["Update", "Merit", "Gestation Time", "Fitness", "Repro Rate?", "(deprecated) Size",
                "Copied Size", "Executed Size", "(deprecated) Abundance",
                "Proportion of organisms that gave birth in this update", "Proportion of Breed True Organisms",
                "(deprecated) Genotype Depth", "Generation", "Neutral Metric", "Lineage Label",
                "True Replication Rate (based on births/update, time-averaged)"]
TIME_COLS = ["update", "avida time", "average generation", "num_executed?"]
DOMINANT_COLS = ["Update", "Average Merit of the Dominant Genotype",
                 "Average Gestation Time of the Dominant Genotype",
                 "Average Fitness of the Dominant Genotype", "Repro Rate?", "Size of Dominant Genotype",
                 "Copied Size of Dominant Genotype", "Executed Size of Dominant Genotype",
                 "Abundance of Dominant Genotype", "Number of Births", "Number of Dominant Breed True?",
                 "Dominant Gene Depth", "Dominant Breed In", "Max Fitness?",
                 "Genotype ID of Dominant Genotype", "Name of the Dominant Genotype"]
# count.dat 4 / 5 come from the genotype classification (avida_amd/systematics.py)
# when the driver runs one; dominant.dat 8 is 0 in the reference as well
UNTRACKED = {"count.dat": [11, 12, 13, 16], "average.dat": [5, 6, 11, 14, 15, 16],
             "dominant.dat": [10, 11, 12, 13]}


def fmt(x):
    """cDataFile / ostream default: 6 significant digits"""
    if isinstance(x, (int, str)):
        return str(x)
    return "%g" % x


class DataFile:
    """One reference-style data file: comments, a numbered column legend,
    a blank line, then rows (Avida::Output::File)."""

    def __init__(self, path, comments, columns):
        self.path = path
        self.f = open(path, "w")
        for c in comments:
            self.f.write(f"# {c}\n")
        for i, name in enumerate(columns, 1):
            self.f.write(f"# {i:2d}: {name}\n")
        self.f.write("\n")

    def row(self, values):
        self.f.write(" ".join(fmt(v) for v in values) + " \n")
        self.f.flush()

    def close(self):
        self.f.close()


class StatsRecorder:
    """Keeps what cStats accumulates across updates (avida_time) and writes
    the requested data files from avgpu_update_stats."""

    def __init__(self, data_dir, resource_names=()):
        self.dir = data_dir
        os.makedirs(data_dir, exist_ok=True)
        self.files = {}
        self.avida_time = 0.0
        self.last = None
        self.resource_names = list(resource_names)
        self.arbiter = None       # systematics.GenotypeArbiter, set by the driver
        self.injected = 0         # organisms injected / loaded in the current update

    def _stamp(self):
        return time.strftime("%a %b %d %H:%M:%S %Y")

    def _file(self, name, comments, cols):
        if name not in self.files:
            self.files[name] = DataFile(os.path.join(self.dir, name), comments, cols)
        return self.files[name]

    def begin_update(self):
        """cStats::ProcessUpdate at the start of an update > 0: avida time
        advances by 1 / (average merit at the end of the previous update)"""
        s = self.last
        if s is not None and s.num_organisms > 0 and s.sum_merit > 0:
            self.avida_time += 1.0 / (s.sum_merit / s.num_organisms)

    def end_update(self, stats):
        """the reference counts injected and loaded organisms as births of the
        update they arrive in (cPopulation::ActivateOrganism -> cStats
        RecordBirth, main/cPopulation.cc:1320-1340)"""
        if self.injected:
            stats.births += self.injected
            self.injected = 0
        self.last = stats

    def print_count(self, name="count.dat"):
        s = self.last
        n = s.num_organisms
        f = self._file(name, ["Avida count data", self._stamp()], COUNT_COLS)
        a = self.arbiter
        ng, nt = (a.num_genotypes(), a.num_threshold()) if a is not None else (0, 0)
        f.row([s.update, s.insts_executed - s.insts_wasted, n, ng, nt, 0, 0, 0, s.births, s.deaths, 0, 0, 0, n, 0, 0])

    def print_dominant(self, name="dominant.dat"):
        """cActionPrintDominantData (actions/PrintActions.cc:5405-5440): the
        file is opened on the first call; with no organism no row is written"""
        f = self._file(name, ["Avida Dominant Data", self._stamp()], DOMINANT_COLS)
        row = self.arbiter.dominant_row(self.last.update) if self.arbiter is not None else None
        if row is not None:
            f.row(row)

    def print_average(self, name="average.dat"):
        s = self.last
        n = s.num_organisms
        avg = (lambda v: v / n) if n else (lambda v: 0.0)
        f = self._file(name, ["Avida Average Data", self._stamp()], AVERAGE_COLS)
        copied = executed = 0.0
        c = self.arbiter.census if self.arbiter is not None else None
        if c is not None and n:                     # cStats copied / executed size sums
            live = c["genotype_key"] != 0
            copied = float(c["copied_size"][live].astype("f8").sum()) / n
            executed = float(c["executed_size"][live].astype("f8").sum()) / n
        f.row([s.update, avg(s.sum_merit), avg(s.sum_gestation), avg(s.sum_fitness), 0, 0, copied, executed, 0,
               (s.births / n) if n else 0.0, 0, 0, s.ave_generation, 0, 0, 0])

    def print_tasks(self, name="tasks.dat"):
        s = self.last
        f = self._file(name, ["Avida tasks data", self._stamp(),
                              "First column gives the current update, next columns give the number",
                              "of organisms that have the particular task as a component of their merit"],
                       ["Update"] + TASK_NAMES)
        f.row([s.update] + [int(s.task_orgs[t]) for t in range(9)])

    def print_time(self, name="time.dat"):
        s = self.last
        f = self._file(name, ["Avida time data", self._stamp()], TIME_COLS)
        f.row([s.update, self.avida_time, s.ave_generation, s.insts_executed - s.insts_wasted])

    def print_resource(self, levels, name="resource.dat"):
        f = self._file(name, ["Avida resource data", self._stamp(),
                              "First column gives the current update, all further columns give the quantity",
                              "of the particular resource at that update."],
                       ["Update"] + self.resource_names)
        f.row([self.last.update] + list(levels))

    def close(self):
        for f in self.files.values():
            f.close()
