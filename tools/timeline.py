"""One update's kernel timeline from a rocprofv3 kernel trace (diagnostic):
  python tools/timeline.py gpurun_out/prof_X/run_kernel_trace.csv [step]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 15
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    c0 = [i for i, r in enumerate(rows) if ("k_interpret<316" in r["Kernel_Name"] or "k_interpret<320" in r["Kernel_Name"])]
    t0 = int(rows[c0[step - 1]]["End_Timestamp"])
    tail = 0
    for r in rows[c0[step - 1] + 1:c0[step] + 1]:
        s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        print("%8.1f %8.1f %7.1f q%s %s" % (s / 1e3, e / 1e3, (e - s) / 1e3, r["Queue_Id"], r["Kernel_Name"][:70]))
    print("c0 start after previous c0 end: %.1f us" % ((int(rows[c0[step]]["Start_Timestamp"]) - t0) / 1e3))


if __name__ == "__main__":
    main()
