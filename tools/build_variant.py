"""Build an A/B variant of the product library (diagnostics, never shipped as
the product): a copy of avida_amd/csrc with text substitutions applied,
compiled to avida_amd/libavida_gpu_<NAME>.so, which bench.py loads when
AVGPU_DIAG_LIB points at it (tools/gpu/ab_var.sh).
usage: python tools/build_variant.py NAME 'FILE:OLD=>NEW' ..."""
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from avida_amd import build as b  # noqa: E402


def main():
    name, subs = sys.argv[1], sys.argv[2:]
    tmp = tempfile.mkdtemp(prefix="var_" + name + "_")
    src = os.path.join(tmp, "avida_amd", "csrc")
    shutil.copytree(b.CSRC, src)
    os.makedirs(os.path.join(tmp, "include"))
    shutil.copy(os.path.join(ROOT, "include", "avida_gpu.h"), os.path.join(tmp, "include"))
    for spec in subs:
        f, rest = spec.split(":", 1)
        old, new = rest.split("=>", 1)
        p = os.path.join(src, f)
        text = open(p).read()
        assert old in text, (f, old)
        open(p, "w").write(text.replace(old, new))
    out = os.path.join(b.HERE, f"libavida_gpu_{name}.so")
    cflags = [f for f in b.FLAGS if f != "-shared"]
    objs = [os.path.join(tmp, s + ".o") for s in b.SOURCES]

    def one(k):
        subprocess.run([b.HIPCC, *cflags, "-c", "-o", objs[k], os.path.join(src, b.SOURCES[k])], check=True)

    with ThreadPoolExecutor(len(b.SOURCES)) as ex:
        list(ex.map(one, range(len(b.SOURCES))))
    subprocess.run([b.HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out, *objs], check=True)
    shutil.rmtree(tmp)
    print(out)


if __name__ == "__main__":
    main()
