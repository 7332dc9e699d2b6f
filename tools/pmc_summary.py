"""Average rocprofv3 --pmc counters per dispatch for kernels matching a regex.

usage: python tools/pmc_summary.py 'gpurun_out/pmc_TAG_*/**/*counter_collection.csv' [regex]
       [--json OUT --world 1024x1024 --source TEXT]

With --json, also writes the HBM traffic per launch of the matched kernel
(MI355X_MICROARCH.md "HBM": FETCH_SIZE on gfx950 reports half of the bytes of
a coalesced read, so traffic = 2 * FETCH_SIZE + WRITE_SIZE; both in KiB)."""
import argparse
import csv
import glob
import json
import re
from collections import defaultdict


# the class-0 main pass (its last template flag, NB, false; the newborn pass
# is the same kernel with NB = true: tools/pmc_summary.py PATTERN NB_REGEX)
MAIN = r"k_interpret<(316|320),[^(]*false>\("
NB_REGEX = r"k_interpret<(316|320),[^(]*true>\("


def summarize(pattern, regex=MAIN, last=0):
    """per counter, the average over the matching dispatches (last > 0: each
    file's last `last` of them by dispatch id -- the bench's warmup and timed
    updates, not the burn-in, whose lock-step first updates take more batch
    steps of fewer instructions each)"""
    vals = defaultdict(list)
    for f in sorted(glob.glob(pattern, recursive=True)):
        per = defaultdict(list)
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if not re.search(regex, row.get("Kernel_Name", "")):
                    continue
                per[row["Counter_Name"]].append((int(row["Dispatch_Id"]), float(row["Counter_Value"])))
        for k, v in per.items():
            v.sort()
            vals[k].extend(x for _, x in (v[-last:] if last > 0 else v))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("pattern")
    ap.add_argument("regex", nargs="?", default=MAIN)
    ap.add_argument("--json")
    ap.add_argument("--world", default="1024x1024")
    ap.add_argument("--source", default="")
    ap.add_argument("--last", type=int, default=0, help="each file's last N matching dispatches only")
    a = ap.parse_args()
    avg, n = summarize(a.pattern, a.regex, a.last)
    for k in sorted(avg):
        print("%-28s %18.1f  (n=%d)" % (k, avg[k], n[k]))
    if a.json:
        fetch = avg.get("FETCH_SIZE", 0.0) * 1024.0
        write = avg.get("WRITE_SIZE", 0.0) * 1024.0
        import os
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from avida_amd import capi
        # the library build the counters belong to: bench.py pairs them only
        # with timings of the same build
        out = {"kernel": a.regex, "world": a.world, "source": a.source, "lib_sha16": capi.lib_build_hash(),
               "fetch_size_bytes": fetch, "write_size_bytes": write,
               "hbm_bytes_per_launch": 2.0 * fetch + write,
               "counters_per_dispatch": avg}
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
