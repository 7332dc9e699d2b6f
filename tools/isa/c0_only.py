"""Write a trimmed copy of interp.hip that instantiates only the class-0
world kernel of the bench (REC, C0W, SIMPLE, DEF), for fast ISA / register-count experiments:

  python tools/isa/c0_only.py /tmp/isa/c0.hip [extra #define lines...]
  hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off \
      -I avida_amd/csrc --offload-device-only -S -o /tmp/isa/c0.s /tmp/isa/c0.hip
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
src = open(os.path.join(ROOT, "avida_amd", "csrc", "interp.hip")).read()
cut = src.index("}  // namespace\n")
body = src[:cut]
tail = """
void c0_launch(const DevWorld* dW) {
  hipLaunchKernelGGL((k_interpret<CLASS0_SIZE, true, true, true, true, false>), dim3(1), dim3(64), 0, 0, dW, 0, 0,
                     (int)AVGPU_MODE_WORLD, (int64_t)0, (int64_t)0, 1, 64, 0);
}
}  // namespace
void c0_entry(const DevWorld* dW) { c0_launch(dW); }
"""
defs = "".join("#define %s\n" % d.replace("=", " ", 1) for d in sys.argv[2:])
open(sys.argv[1], "w").write(defs + body + tail)
