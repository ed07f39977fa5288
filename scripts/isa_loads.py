#!/usr/bin/env python3
"""Per-kernel global-load / wait statistics of a gfx950 assembly dump:
flags kernels whose loads are serialised by s_waitcnt vmcnt(0)."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "whisper.rs_amd/csrc/wmi_kernels.hip"
asm = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                      "--offload-device-only", "-S", "-o", "-", src], capture_output=True, text=True, check=True).stdout
dem = {}
for m in re.finditer(r"^(_Z\w+):", asm, re.M):
    name = m.group(1)
    end = asm.find("s_endpgm", m.end())
    body = asm[m.end():end]
    loads = len(re.findall(r"\b(global|buffer)_load", body))
    waits0 = len(re.findall(r"s_waitcnt vmcnt\(0\)", body))
    # loads immediately followed (within 2 lines) by a full wait
    ser = len(re.findall(r"(?:global|buffer)_load[^\n]*\n(?:[^\n]*\n)?\s*s_waitcnt vmcnt\(0\)", body))
    dem[name] = (loads, waits0, ser)
names = subprocess.run(["c++filt"], input="\n".join(dem), capture_output=True,
                       text=True).stdout.split("\n")
for (k, (l, w, s)), n in zip(dem.items(), names):
    if "dec" in n or "attn" in n or "--all" in sys.argv:
        print(f"{l:5d} loads {w:4d} vmcnt(0) {s:4d} serialised  {n[:90]}")
