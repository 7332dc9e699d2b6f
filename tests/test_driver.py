"""The Avida2Driver restatement (avida_amd/driver.py) on a reference test's
config directory (tests/golden/spatial_res_100u/config: avida.cfg,
events.cfg, environment.cfg, the legacy instruction set, the ancestor) writes
the reference's data files: same header comments and column legends, and
where the values do not depend on the reference's RNG stream, the same
numbers (update 0: 100 injected organisms, ResA 20 and the global pool
98.5913; the never-consumed global pool at every printed update).  Update 0's
instruction count is 3000 in the reference, whose scheduler draws UD = 30 x 100
picks; the batch update splits exactly UD picks down its multinomial tree
(DESIGN.md 5), so every update executes AVE_TIME_SLICE x (organisms at its
start) instructions -- 3000 at update 0 -- with one batch step or with
sub-updates (the steps' shares sum to UD).  Later updates can fall short of
it by the picks an organism still had when it died in its slice (AGE_LIMIT):
the reference gives those picks to the living, the batch budgets were drawn
at the update's start.
Update 0's births / deaths differ by design: the reference counts the 101
injections as births (and the replaced first organism as a death)."""
import os

import pytest

from avida_amd import datafiles, driver
import oracle_lib as ol


def _rows(path):
    return {int(l.split()[0]): l.split()[1:] for l in open(path) if l.strip() and not l.startswith("#")}


def _header(path):
    return [l for l in open(path) if l.startswith("#")][2:]   # after the title and the time stamp


@pytest.mark.parametrize("sub_updates", [0, 1, 3])
def test_driver_spatial_res_100u(golden, tmp_path, sub_updates):
    ref = os.path.join(golden, "spatial_res_100u")

    def mk(cfg, iset, env):
        cfg.sub_updates = sub_updates
        return ol.Backend("oracle", cfg, iset, env)
    d = driver.Driver(os.path.join(ref, "config"), str(tmp_path), make_world=mk)
    last = d.run()
    assert last == 100                                  # "u 100 Exit"
    for name in ("count.dat", "average.dat", "tasks.dat", "time.dat", "resource.dat"):
        assert _header(os.path.join(tmp_path, name)) == _header(os.path.join(ref, name)), name
        assert sorted(_rows(os.path.join(tmp_path, name))) == list(range(0, 101, 10)), name
    res, want = _rows(os.path.join(tmp_path, "resource.dat")), _rows(os.path.join(ref, "resource.dat"))
    assert res[0][0] == want[0][0]                      # ResA
    assert [res[u][2] for u in range(0, 101, 10)] == [want[u][2] for u in range(0, 101, 10)]
    cnt, wcnt = _rows(os.path.join(tmp_path, "count.dat")), _rows(os.path.join(ref, "count.dat"))
    assert cnt[0][1] == wcnt[0][1]                      # organisms
    assert int(cnt[0][0]) == int(wcnt[0][0]) == 3000    # insts executed: exactly UD
    # later updates: the allotment's UD less the newborns' carry, plus the
    # newborns' own picks, less what the organisms they replaced ran after
    # their births: UD again, up to the carry still pending
    assert all(int(r[0]) <= 3150 for r in cnt.values())
    tasks = _rows(os.path.join(tmp_path, "tasks.dat"))
    assert tasks[0] == ["0"] * 9
    time_ = _rows(os.path.join(tmp_path, "time.dat"))
    assert time_[0][:2] == ["0", "0"] and int(time_[0][2]) == int(cnt[0][0])


def test_datafile_format(tmp_path):
    f = datafiles.DataFile(os.path.join(tmp_path, "x.dat"), ["Avida x data"], ["update", "value"])
    f.row([0, 1.0])
    f.row([10, 2.0 / 3.0])
    f.close()
    assert open(os.path.join(tmp_path, "x.dat")).read() == \
        "# Avida x data\n#  1: update\n#  2: value\n\n0 1 \n10 0.666667 \n"
