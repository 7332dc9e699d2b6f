"""Per-instruction traces of the GPU interpreter in the reference's format.

The reference's tracer (cHardwareTracer, driven from SingleProcess right
before each instruction executes, cpu/cHardwareCPU.cc:956) prints
cHardwareCPU::PrintStatus (cpu/cHardwareCPU.cc:1111-1169) for every cycle:

    <cpu cycles> IP:<ip> (<instruction name>)
    AX:<v> [0x<hex>]  BX:<v> [0x<hex>]  CX:<v> [0x<hex>]  [  EnergyUsed:<time used>]
      R-Head:<r> W-Head:<w> F-Head:<f>  RL:<read label>
    * Stack 0: Ox<8 hex> x 10          (the current stack starred, top first)
      Stack 1: Ox<8 hex> x 10
      Mem (<size>):  <instruction symbols>

`status_text` formats one avgpu_get_states record (+ its memory), taken
before an instruction, as the tracer sees it: SingleProcess has already
counted the cycle (:929-930) and adjusted the IP (:952) when it calls the
tracer (:956).  `trace` steps a range of cells one instruction at a time through the
C-ABI (avgpu_step, budget 1) and returns the status of every organism before
every instruction -- the GPU-side equivalent of running the reference with a
trace file.  Command line:

    python -m avida_amd.trace -c <config dir or tests/golden> -g <org file> -n 400
"""
from __future__ import annotations

import argparse
import ctypes as C
import os

from avida_amd import capi, files

STACK_SIZE = capi.STACK_SIZE


def _adjust(pos, size):
    """cHeadCPU::Adjust (cpu/cHeadCPU.cc:27-50)"""
    if 0 <= pos < size:
        return pos
    if size == 0 or pos < 0:
        return 0
    if pos < 2 * size:
        return pos - size
    return pos % size


def _hex32(v):
    return "%x" % (v & 0xFFFFFFFF)


def status_text(st, ops, iset: files.InstSet) -> str:
    """cHardwareCPU::PrintStatus of one state record; `ops` = memory op codes"""
    m = st.mem_size
    ip = _adjust(st.head[0], m)
    name = iset.names[ops[ip]] if m else "(none)"
    lines = [f"{st.cpu_cycles_used + 1} IP:{ip} ({name})"]
    regs = "".join(f"{chr(ord('A') + i)}X:{st.reg[i]} [0x{_hex32(st.reg[i])}]  " for i in range(3))
    if st.time_used != st.cpu_cycles_used:
        regs += f"  EnergyUsed:{st.time_used + 1}"
    lines.append(regs)
    label = "".join(chr(ord("A") + st.read_label[k]) for k in range(st.read_label_len))
    lines.append(f"  R-Head:{st.head[1]} W-Head:{st.head[2]} F-Head:{st.head[3]}  RL:{label}   ")
    for k in range(2):
        sp = st.stack_ptr[k]
        vals = [st.stack[k][(sp + d) % STACK_SIZE] for d in range(STACK_SIZE)]   # cCPUStack::Get(depth)
        star = "*" if st.cur_stack == k else " "
        lines.append(f"{star} Stack {k}:" + "".join(" Ox%08x" % (v & 0xFFFFFFFF) for v in vals))
    lines.append(f"  Mem ({m}):  " + iset.to_sequence(ops[:m]))
    return "\n".join(lines) + "\n"


def trace(lib, handle, first, count, n_instructions, iset, mode=capi.MODE_FROZEN, cap=capi.MAX_GENOME):
    """Status texts [step][organism] before each of n_instructions single
    instructions of cells first .. first+count-1 (avgpu_step, budget 1)."""
    out = []
    st = (capi.AvgpuCpuState * count)()
    ops = (C.c_uint8 * (count * cap))()
    fl = (C.c_uint8 * (count * cap))()
    for _ in range(n_instructions):
        capi.check(lib, lib.avgpu_get_states(handle, first, count, st, ops, fl, cap))
        raw = bytes(ops)
        out.append([status_text(st[i], raw[i * cap:(i + 1) * cap], iset) for i in range(count)])
        capi.check(lib, lib.avgpu_step(handle, first, count, None, 1, mode))
    capi.check(lib, lib.avgpu_sync(handle))
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("-c", "--config", default=os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "tests", "golden"))
    ap.add_argument("-g", "--genome", default="default-heads.org")
    ap.add_argument("-i", "--instset", default="instset-heads.cfg")
    ap.add_argument("-n", type=int, default=400)
    ap.add_argument("-o", "--out", default="-")
    args = ap.parse_args()
    iset = files.read_instset(os.path.join(args.config, args.instset))
    env = files.read_environment(os.path.join(args.config, "environment-logic9.cfg"))
    cfg = capi.cfg_from_avida(files.read_avida_cfg(None, {"COPY_MUT_PROB": 0.0, "DIVIDE_INS_PROB": 0.0,
                                                          "DIVIDE_DEL_PROB": 0.0}))
    genome = files.read_org(os.path.join(args.config, args.genome), iset)
    lib = capi.load_product()
    h = lib.avgpu_create(C.byref(cfg), 0, 1)
    if not h:
        raise SystemExit(lib.avgpu_last_error().decode())
    hid = (C.c_uint8 * len(iset.names))(*iset.handlers)
    red = (C.c_int32 * len(iset.names))(*iset.redundancy)
    capi.check(lib, lib.avgpu_load_instset(h, len(iset.names), hid, red))
    arr = capi.reactions_array(env)
    capi.check(lib, lib.avgpu_load_env(h, len(env), arr))
    buf = (C.c_uint8 * len(genome)).from_buffer_copy(genome)
    lens = (C.c_int32 * 1)(len(genome))
    capi.check(lib, lib.avgpu_set_orgs(h, 0, 1, buf, lens, None, None, 1))   # test-CPU inputs
    steps = trace(lib, h, 0, 1, args.n, iset)
    text = "".join(s[0] for s in steps)
    if args.out == "-":
        print(text, end="")
    else:
        with open(args.out, "w") as f:
            f.write(text)
    lib.avgpu_destroy(h)


if __name__ == "__main__":
    main()
