"""Per-kernel VGPR / spill counts of a HIP source for gfx950 (device-only asm, no GPU needed).
usage: python tools/isa_regs.py dune-pnp_amd/csrc/assemble.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
out = "/tmp/isa_regs.s"
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950",
                       "--cuda-device-only", "-S", "-o", out, src], stderr=subprocess.DEVNULL)
txt = open(out).read()
meta = txt[txt.index("amdhsa.kernels"):]
for blk in re.split(r"\n  - ", meta)[1:]:
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    name = subprocess.run(["c++filt"], input=g("name"), capture_output=True, text=True).stdout.strip()
    if filt in name:
        print(f"vgpr={g('vgpr_count'):>4} spill={g('vgpr_spill_count'):>3} "
              f"lds={g('group_segment_fixed_size'):>6}  {name[:110]}")
