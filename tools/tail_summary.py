"""Per-update breakdown of the time outside class 0 (diagnostic), from a
rocprofv3 kernel trace: python tools/tail_summary.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # anchors: the class-0 main pass (the newborn pass, template flag NB = true,
    # is a tail item of its own)
    def main_pass(r):
        n = r["Kernel_Name"]
        return ("k_interpret<316" in n or "k_interpret<320" in n) and not n.split("(DevWorld")[0].endswith("true>")
    idx = [i for i, r in enumerate(rows) if main_pass(r)]
    acc = defaultdict(float)
    gaps = aux_over = 0.0
    steps = 0
    for a, b in zip(idx[-41:-1], idx[-40:]):
        c0_end = int(rows[a]["End_Timestamp"])
        t = c0_end
        for r in rows[a + 1:b]:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if r["Queue_Id"] != rows[a]["Queue_Id"]:
                if s < c0_end:
                    aux_over = max(aux_over, 0)
                continue
            gaps += max(0, s - t) / 1e3
            name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if name.startswith("k_interpret<316") or name.startswith("k_interpret<320"):
                name = "newborn pass " + name
            elif name.startswith("k_interpret"):
                name = ("newborn " if name.endswith("true>") else "") + "spill " + name
            if name == "k_place_pick_mut":   # the split diagnostic build launches its parts apart
                name += " [%d blocks]" % (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]))
            acc[name] += (e - s) / 1e3
            t = e
        gaps += max(0, int(rows[b]["Start_Timestamp"]) - t) / 1e3
        steps += 1
    tot = sum(acc.values()) + gaps
    for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
        print("%-40s %7.1f us/update" % (k, v / steps))
    print("%-40s %7.1f us/update" % ("gaps (incl. waits for aux streams)", gaps / steps))
    print("%-40s %7.1f us/update" % ("total outside the class-0 main pass", tot / steps))


if __name__ == "__main__":
    main()
