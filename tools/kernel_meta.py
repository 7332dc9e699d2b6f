"""Per-kernel register / LDS / scratch metadata of the gfx950 code object in
libavida_gpu.so (diagnostic): the .hip_fatbin section's offload bundle is
unpacked and its AMDGPU metadata notes read with llvm-readelf.

usage: python tools/kernel_meta.py [lib.so] [name-filter]"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(path):
    data = open(path, "rb").read()
    pos = 0
    while True:
        pos = data.find(MAGIC, pos)
        if pos < 0:
            return
        n, = struct.unpack_from("<Q", data, pos + 24)
        q = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, q)
            triple = data[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if "gfx950" in triple:
                yield data[pos + off:pos + off + size]
        pos += 24


def kernels(path):
    out = []
    for co in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
        cur = {}
        for line in notes.splitlines():
            m = re.match(r"\s+\.(\w+):\s+(.*)", line)
            if not m:
                continue
            k, v = m.group(1), m.group(2).strip()
            if k == "name" and "_ZN" in v or (k == "name" and v.startswith("_Z")):
                cur = {"name": v}
                out.append(cur)
            elif k in ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
                       "private_segment_fixed_size", "group_segment_fixed_size"):
                cur[k] = int(v)
    return out


def demangle(names):
    r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    return r.stdout.splitlines()


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "avida_amd", "libavida_gpu.so")
    flt = sys.argv[2] if len(sys.argv) > 2 else "k_interpret"
    ks = kernels(lib)
    names = demangle([k["name"] for k in ks])
    for k, nm in zip(ks, names):
        if flt not in nm:
            continue
        nm = re.sub(r"\(anonymous namespace\)::", "", nm)
        nm = nm.split("(")[0]
        print(f"{k.get('vgpr_count', -1):4d} v {k.get('agpr_count', 0):3d} a {k.get('sgpr_count', -1):3d} s "
              f"spill v{k.get('vgpr_spill_count', 0)} s{k.get('sgpr_spill_count', 0)} "
              f"scratch {k.get('private_segment_fixed_size', 0):5d} lds {k.get('group_segment_fixed_size', 0):6d}  {nm}")


if __name__ == "__main__":
    main()
