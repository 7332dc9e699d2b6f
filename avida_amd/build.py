"""Build the in-tree HIP library avida_amd/libavida_gpu.so for gfx950.

hipcc cross-compiles without a GPU; the .so travels to the GPU box with the
repository snapshot (it is git-ignored, not gpurun-ignored).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
SOURCES = ["interp.hip", "world.hip", "resources.hip", "capi.hip"]
OUT = os.path.join(HERE, "libavida_gpu.so")
# diagnostic variant with per-phase s_memtime clocks (tools/phase_clocks.py only)
OUT_CLK = os.path.join(HERE, "libavida_gpu_clk.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "--offload-arch=gfx950", "-std=c++17", "-fPIC", "-shared",
         "-ffp-contract=off", "-Wno-unused-result", "-Wno-unused-value"]


def needs_build(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(ROOT, "include", "avida_gpu.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, clocks: bool = False) -> str:
    """Each source compiled on its own (in parallel), then one shared link."""
    from concurrent.futures import ThreadPoolExecutor
    out = OUT_CLK if clocks else OUT
    if not force and not needs_build(out):
        return out
    extra = ["-DAVGPU_PHASE_CLOCKS"] if clocks else []
    cflags = [f for f in FLAGS if f != "-shared"]
    objs = [out + "." + os.path.splitext(src)[0] + ".o" for src in SOURCES]

    def compile_one(k):
        cmd = [HIPCC, *cflags, *extra, "-c", "-o", objs[k], os.path.join(CSRC, SOURCES[k])]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)

    with ThreadPoolExecutor(len(SOURCES)) as ex:
        list(ex.map(compile_one, range(len(SOURCES))))
    cmd = [HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "-o", out + ".tmp", *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
    os.replace(out + ".tmp", out)
    return out


# the C++ host driver of strip-tiled worlds (RCCL between ranks)
HOST_SRC = os.path.join(HERE, "host", "strips.cc")
HOST_OUT = os.path.join(HERE, "bin", "avgpu_strips")


def build_host(force: bool = False, verbose: bool = False) -> str:
    lib = build(force=False, verbose=verbose)
    if not force and os.path.exists(HOST_OUT) and \
            os.path.getmtime(HOST_OUT) > max(os.path.getmtime(HOST_SRC), os.path.getmtime(lib)):
        return HOST_OUT
    os.makedirs(os.path.dirname(HOST_OUT), exist_ok=True)
    cmd = [HIPCC, "-O2", "-std=c++17", "-Wno-unused-result", "-I", os.path.join(ROOT, "include"),
           "-o", HOST_OUT + ".tmp", HOST_SRC, "-L", HERE, "-lavida_gpu", "-lrccl",
           "-Wl,-rpath,$ORIGIN/..", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(HOST_OUT + ".tmp", HOST_OUT)
    return HOST_OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True, clocks="--clocks" in sys.argv)
    build_host(force="--force" in sys.argv, verbose=True)
