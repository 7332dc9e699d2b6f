"""HBM roofline of the resource step (configs[4]) from a rocprofv3 kernel-stats
CSV of `bench.py --env resources`: k_res_step moves 16 algorithmic bytes per
cell and spatial resource (the amount read, the next amount written;
neighbours come from L2), one launch per update for all of the resources
(DESIGN.md section 7).
usage: python tools/res_roofline.py run_kernel_stats.csv side n_resources [peak_GBs]"""
import csv
import json
import re
import sys


def main():
    path, side, nres = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    peak = float(sys.argv[4]) if len(sys.argv) > 4 else 8000.0
    cells = side * side
    rows = {r["Name"]: r for r in csv.DictReader(open(path))}
    out = {}
    for name, r in rows.items():
        if "k_res_step" not in name:
            continue
        avg_ns = float(r["AverageNs"])
        b = 16.0 * cells * nres
        gbs = b / (avg_ns * 1e-9) / 1e9
        key = re.search(r"k_res_step\w*(<[^>]*>)?", name).group(0)
        out[key] = {
            "calls": int(r["Calls"]), "avg_us": avg_ns / 1e3, "bytes_per_launch": b,
            "achieved_GBs": gbs, "peak_GBs": peak, "frac": gbs / peak}
    print(json.dumps({"cells": cells, "resources": nres, "k_res_step": out}, indent=1))


if __name__ == "__main__":
    main()
