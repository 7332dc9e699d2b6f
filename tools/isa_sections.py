"""Static instruction mix per marked section of one interpreter kernel.

Build the marked assembly first (markers are `asm volatile` comments at the
phase-clock points of interp.hip, compiled only with -DAVGPU_ISA_MARKS):

  hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off \
      -DAVGPU_ISA_MARKS --offload-device-only -S -o marks.s avida_amd/csrc/interp.hip
  python tools/isa_sections.py marks.s [320] [0] [Lb1ELb1ELb1]

Counts are static (instructions between a marker and the next one in layout
order), not executed counts: a section the compiler splits across blocks is
summed over its pieces."""
import re
import sys


def classify(line):
    if not line or line.startswith((";", ".")) or line.endswith(":"):
        return None
    op = line.split()[0]
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch")):
        return "br"
    if op.startswith(("s_load", "s_buffer", "s_memtime")):
        return "smem"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("scratch_"):
        return "scratch"
    return "other"


def main():
    path = sys.argv[1]
    size = sys.argv[2] if len(sys.argv) > 2 else "320"
    rec = sys.argv[3] if len(sys.argv) > 3 else "0"
    flags = sys.argv[4] if len(sys.argv) > 4 else ""   # e.g. "Lb1ELb1ELb1" for the C0W/SIMPLE/DEF kernel
    text = open(path).read()
    m = re.search(r"^(_Z\S*k_interpretILi%sELb%sE%s\S*):" % (size, rec, flags), text, re.M)
    body = text[m.end():]
    body = body[:body.index(".Lfunc_end")]
    cur, stats, total = "entry", {}, {}
    for raw in body.split("\n"):
        line = raw.strip()
        mm = re.search(r"@MARK (\S+)", line)
        if mm:
            cur = mm.group(1)
            continue
        c = classify(line)
        if c:
            stats.setdefault(cur, {})
            stats[cur][c] = stats[cur].get(c, 0) + 1
            total[c] = total.get(c, 0) + 1
    keys = ["valu", "salu", "lds", "vmem", "scratch", "smem", "wait", "br", "other"]
    print("%-8s" % "section" + "".join("%8s" % k for k in keys) + "%8s" % "all")
    for sec, v in stats.items():
        print("%-8s" % sec + "".join("%8d" % v.get(k, 0) for k in keys) + "%8d" % sum(v.values()))
    print("%-8s" % "total" + "".join("%8d" % total.get(k, 0) for k in keys) + "%8d" % sum(total.values()))


if __name__ == "__main__":
    main()
