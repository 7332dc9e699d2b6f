"""bench.py --gpus N without torch.distributed.run starts the N ranks itself
(bench.relaunch_ranks) -- rehearsed here on the CPU: 2 gloo ranks of the
oracle strip world (tests/bench_rank_oracle.py) launched through the same
torch.distributed.run command, whose states must equal the untiled world."""
import json
import os
import subprocess
import sys

import pytest
import torch

import bench
from avida_amd import capi
import parity_util as pu
import tile_util as tu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_rank_env_rejects_mismatched_world(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    assert bench.rank_env(4) == (1, 4, 1)
    with pytest.raises(SystemExit):
        bench.rank_env(8)


def test_relaunch_two_gloo_ranks_equal_single_world(golden, tmp_path, capfd):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["OMP_NUM_THREADS"] = "1"
    rc = bench.relaunch_ranks(2, ["--gpus", "2", "--updates", "12", "--out", str(tmp_path)],
                              script=os.path.join(HERE, "bench_rank_oracle.py"), env=env)
    out = capfd.readouterr().out
    assert rc == 0, out
    line = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert line["ranks"] == 2
    X, Y, T = 32, 32, 2
    ref, _ = tu.single("oracle", golden, X, Y, 12)
    a, oa, fa = ref.states(0, X * Y, 512)
    per = X * Y // T
    for k in range(T):
        d = torch.load(os.path.join(tmp_path, f"rank{k}.pt"), weights_only=True)
        s = (capi.AvgpuCpuState * per).from_buffer_copy(d["states"])
        lo = k * per
        bad = pu.diff_states(a[lo:lo + per], s, oa[lo * 512:(lo + per) * 512], d["ops"],
                             fa[lo * 512:(lo + per) * 512], d["flags"], 512)
        assert not bad, f"rank {k}: {bad[:3]}"
    assert line["births"] > 0
