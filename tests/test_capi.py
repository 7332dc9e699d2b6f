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


# (avgpu_cfg field, value away from the reference default) for every knob of
# the refused block and every value outside an implemented range: the C-ABI
# itself must refuse each (avgpu_check_cfg / avgpu_create -> AVGPU_EUNSUPPORTED)
REFUSED_C = [
    ("point_mut_prob", "0.01"), ("point_ins_prob", "0.01"), ("point_del_prob", "0.01"),
    ("inst_point_mut_prob", "0.01"), ("div_lgt_prob", "0.01"), ("divide_lgt_prob", "0.01"),
    ("divide_poisson_lgt_mean", "1.0"), ("inject_mut_prob", "0.01"), ("inject_ins_prob", "0.01"),
    ("inject_del_prob", "0.01"), ("meta_copy_mut", "0.1"), ("meta_std_dev", "0.1"),
    ("death_prob", "0.1"), ("age_deviation", "3"), ("divide_failure_resets", "1"),
    ("special_mut_line", "5"), ("population_cap", "100"), ("generation_inc_method", "0"),
    ("reset_inputs_on_divide", "1"), ("epigenetic_method", "1"), ("min_cycles", "10"),
    ("required_task", "16"), ("immunity_task", "16"), ("required_reaction", "12"),
    ("immunity_reaction", "12"),
    ("require_exact_copy", "1"), ("fitness_method", "1"), ("juv_period", "5"),
    ("no_mut_insts_len", "1"), ("test_fitness_measures", "1"),
    ("divide_method", "0"), ("world_geometry", "3"), ("slicing_method", "3"),
    ("base_merit_method", "6"), ("birth_method", "6"), ("death_method", "3"), ("alloc_method", "1"),
    ("sub_updates", "65"),
]


def test_c_abi_refuses_every_unimplemented_knob(tmp_path):
    """Each knob set through the compiled header is refused by the library
    (avgpu_check_cfg, the check avgpu_create runs first), naming the knob; the
    defaults are accepted."""
    build.build()
    body = "\n".join(
        f'  {{ avgpu_cfg c; avgpu_cfg_defaults(&c); c.{f} = {v}; int rc = avgpu_check_cfg(&c);'
        f' printf("{f} %d %s\\n", rc, avgpu_last_error()); }}' for f, v in REFUSED_C)
    src = tmp_path / "refuse.c"
    src.write_text('#include "avida_gpu.h"\n#include <stdio.h>\nint main(void){\n'
                   '  { avgpu_cfg c; avgpu_cfg_defaults(&c); printf("defaults %d\\n", avgpu_check_cfg(&c)); }\n'
                   + body + "\n  return 0;\n}\n")
    exe = tmp_path / "refuse"
    libdir = os.path.dirname(capi.LIB_PATH)
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe), "-L", libdir,
                    "-lavida_gpu", f"-Wl,-rpath,{libdir}"], check=True)
    lines = subprocess.check_output([str(exe)], text=True).strip().split("\n")
    assert lines[0] == "defaults 0"
    got = {ln.split()[0]: ln for ln in lines[1:]}
    for f, _ in REFUSED_C:
        rc = int(got[f].split()[1])
        assert rc == -5, got[f]                      # AVGPU_EUNSUPPORTED
        assert "not on the GPU path" in got[f], got[f]


def test_python_config_reaches_the_refusal(golden, tmp_path):
    """A reference avida.cfg that sets a knob this path does not implement
    fills the avgpu_cfg field, and the library refuses it (no Python-only list)."""
    from avida_amd import files
    lib = capi.load_product()
    for key, field in [("DIV_LGT_PROB", "div_lgt_prob"), ("DIVIDE_POISSON_LGT_MEAN", "divide_poisson_lgt_mean"),
                       ("DIVIDE_LGT_PROB", "divide_lgt_prob"), ("DEATH_PROB", "death_prob"),
                       ("POINT_MUT_PROB", "point_mut_prob")]:
        c = capi.cfg_from_avida(files.read_avida_cfg(None, {key: 0.01}))
        assert getattr(c, field) == 0.01
        assert lib.avgpu_check_cfg(C.byref(c)) == -5
        assert key.split("_")[0] in lib.avgpu_last_error().decode().upper()
    c = capi.cfg_from_avida(files.read_avida_cfg(None, {"STERILIZE_UNSTABLE": 1}))
    assert c.test_fitness_measures == 1 and lib.avgpu_check_cfg(C.byref(c)) == -5
    # NO_MUT_INSTS runs (tests/test_no_mut.py); a length that is not its string's is refused
    c = capi.cfg_from_avida(files.read_avida_cfg(None, {"NO_MUT_INSTS": "abc"}))
    assert c.no_mut_insts_len == 3 and c.no_mut_insts == b"abc" and lib.avgpu_check_cfg(C.byref(c)) == 0
    c.no_mut_insts_len = 4
    assert lib.avgpu_check_cfg(C.byref(c)) == -5
    # SLIP_COPY_MODE 1 (memory slips) runs with fill modes 0 / 2 / 4; 3 and 1 are refused
    for fill, rc in ((0, 0), (2, 0), (4, 0), (3, -5), (1, -5)):
        c = capi.cfg_from_avida(files.read_avida_cfg(None, {"COPY_SLIP_PROB": 0.01, "SLIP_COPY_MODE": 1,
                                                            "SLIP_FILL_MODE": fill}))
        assert lib.avgpu_check_cfg(C.byref(c)) == rc, fill
    # sub-updates need the probabilistic scheduler
    c = capi.cfg_from_avida(files.read_avida_cfg(None, {"SLICING_METHOD": 2}))
    c.sub_updates = 3
    assert lib.avgpu_check_cfg(C.byref(c)) == -5 and "sub_updates" in lib.avgpu_last_error().decode()
    c.slicing_method = 1
    assert lib.avgpu_check_cfg(C.byref(c)) == 0
    # DIV_MUT_PROB (per-site substitutions on divide) is on the path
    c = capi.cfg_from_avida(files.read_avida_cfg(None, {"DIV_MUT_PROB": 0.003}))
    assert c.div_mut_prob == 0.003 and lib.avgpu_check_cfg(C.byref(c)) == 0
    text = open(os.path.join(golden, "avida-default.cfg")).read().replace(
        "POINT_MUT_PROB 0.0", "POINT_MUT_PROB 0.001")
    p = tmp_path / "avida.cfg"
    p.write_text(text)
    c = capi.cfg_from_avida(files.read_avida_cfg(str(p)))
    assert c.point_mut_prob == 0.001 and lib.avgpu_check_cfg(C.byref(c)) == -5
    # the reference's default config itself is accepted
    c = capi.cfg_from_avida(files.read_avida_cfg(os.path.join(golden, "avida-default.cfg")))
    assert lib.avgpu_check_cfg(C.byref(c)) == 0, lib.avgpu_last_error()
