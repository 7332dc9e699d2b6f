"""C-ABI checks that need no GPU: the library builds and loads, exports every
symbol include/avida_gpu.h declares, and the ctypes mirror has the C layout."""
import ctypes as C
import os
import re
import subprocess

import pytest

from avida_amd import capi, build

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "avida_gpu.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(avgpu_[a-z_]+)\s*\(", txt)))


def test_header_and_mirror_agree():
    assert _declared() == sorted(capi.EXPORTED)


def test_library_exports_every_symbol():
    build.build()
    lib = C.CDLL(capi.LIB_PATH)
    missing = [s for s in _declared() if not hasattr(lib, s)]
    assert not missing, missing


def test_struct_layouts(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include "avida_gpu.h"\n#include <stdio.h>\n#include <stddef.h>\n'
                   'int main(){printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(avgpu_cfg),'
                   ' sizeof(avgpu_reaction), sizeof(avgpu_cpu_state), sizeof(avgpu_test_result),'
                   ' sizeof(avgpu_update_stats), offsetof(avgpu_cpu_state, cur_bonus),'
                   ' offsetof(avgpu_cfg, seed)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    exp = [C.sizeof(capi.AvgpuCfg), C.sizeof(capi.AvgpuReaction), C.sizeof(capi.AvgpuCpuState),
           C.sizeof(capi.AvgpuTestResult), C.sizeof(capi.AvgpuUpdateStats),
           capi.AvgpuCpuState.cur_bonus.offset, capi.AvgpuCfg.seed.offset]
    assert got == exp


def test_cfg_defaults_match_avida_cfg(golden):
    from avida_amd import files
    lib = C.CDLL(capi.LIB_PATH)
    c = capi.AvgpuCfg()
    lib.avgpu_cfg_defaults(C.byref(c))
    ref = capi.cfg_from_avida(files.read_avida_cfg(os.path.join(golden, "avida-default.cfg")), seed=101)
    for name, _ in capi.AvgpuCfg._fields_:
        assert getattr(c, name) == getattr(ref, name), name


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = capi.load_product()
    c = capi.AvgpuCfg()
    lib.avgpu_cfg_defaults(C.byref(c))
    h = lib.avgpu_create(C.byref(c), 0, 16)
    assert not h
    assert lib.avgpu_last_error()


def test_unsupported_mutation_knobs_are_refused(golden, tmp_path):
    """A reference avida.cfg that sets a mutation knob this path does not
    implement is refused, not run with different semantics (capi.UNSUPPORTED_NONZERO)."""
    from avida_amd import files
    for key in ["DIV_LGT_PROB", "PARENT_INS_PROB", "DIVIDE_POISSON_LGT_MEAN", "COPY_SLIP_PROB",
                "COPY_UNIFORM_PROB", "DIVIDE_LGT_PROB"]:
        with pytest.raises(ValueError, match=key):
            capi.cfg_from_avida(files.read_avida_cfg(None, {key: 0.01}))
    # DIV_MUT_PROB (per-site substitutions on divide) is on the path
    assert capi.cfg_from_avida(files.read_avida_cfg(None, {"DIV_MUT_PROB": 0.003})).div_mut_prob == 0.003
    text = open(os.path.join(golden, "avida-default.cfg")).read().replace(
        "COPY_SLIP_PROB 0.0", "COPY_SLIP_PROB 0.001")
    p = tmp_path / "avida.cfg"
    p.write_text(text)
    with pytest.raises(ValueError, match="COPY_SLIP_PROB"):
        capi.cfg_from_avida(files.read_avida_cfg(str(p)))
    # the reference's default config itself is accepted
    capi.cfg_from_avida(files.read_avida_cfg(os.path.join(golden, "avida-default.cfg")))
