"""The C++ host driver (avida_amd/host/strips.cc -> avida_amd/bin/avgpu_strips):
the compiled counterpart of avida_amd/tiles.py and bench.py's world setup,
driving the C-ABI with RCCL on the world's stream.  CPU: it is built and
answers --help without touching a GPU.  GPU: T strips exchanging in one
process (loopback) leave every cell of the torus in the same state as the
untiled world (state digests); one rank of independent worlds sharing the
scheduler totals over RCCL equals the untiled world.  (Two RCCL ranks need
two GPUs: the strip exchange over RCCL runs on multi-GPU nodes only.)"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "avida_amd", "bin", "avgpu_strips")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _run(*args, timeout=240):
    out = subprocess.run([BIN, "--config", GOLDEN, *args], capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_host_driver_built():
    assert os.access(BIN, os.X_OK)
    out = subprocess.run([BIN, "--help"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0 and "--strips" in out.stdout


@pytest.mark.gpu
def test_host_driver_strips_equal_untiled():
    common = ["--side", "256", "--updates", "12", "--burn-in", "0", "--seed", "7"]
    flat = _run(*common, "--strips", "2", "--untiled")
    loop = _run(*common, "--strips", "2")
    assert loop["digest_rank0"] == flat["digest_rank0"], (loop, flat)
    assert loop["organisms"] == flat["organisms"]
    # one rank of cMultiProcessWorld-style independent worlds: RCCL all-reduce
    # of the scheduler totals on the world's stream, == the untiled world (one
    # batch step per update: handed-in totals take no adaptive steps)
    one = _run(*common, "--strips", "1", "--untiled", "--sub-updates", "1")
    rccl = _run(*common, "--rccl", "--independent", "--sub-updates", "1")
    assert rccl["ranks"] == 1 and rccl["digest_rank0"] == one["digest_rank0"], (rccl, one)
