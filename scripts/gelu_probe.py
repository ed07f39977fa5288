#!/usr/bin/env python3
"""How often does the device's f32 GELU round to a different f16 than the
host-built ggml table (build_tables in wmi_api.cpp: f16(0.5 f (1 + tanhf(
sqrt(2/pi) f (1 + 0.044715 f f)))) with the host's libm tanhf)?  Evaluates
the same expression, one rounding per operation, for every finite f16 input
on the GPU (torch's f32 tanh: the device math library the kernels call) and
on the host (numpy f32, libm tanhf), and counts the inputs whose f16 results
differ.  A handful would let the GEMM epilogue compute GELU and fall back to
the table only for the listed inputs."""
import numpy as np
import torch

A = np.float32(0.044715)
C = np.float32(0.79788456080286535587989211986876)
H = np.float32(0.5)
ONE = np.float32(1.0)

bits = np.arange(65536, dtype=np.uint16)
f = bits.view(np.float16).astype(np.float32)
fin = np.isfinite(f)
with np.errstate(all="ignore"):
    host = H * f * (ONE + np.tanh(C * f * (ONE + A * f * f)))
host16 = host.astype(np.float16).view(np.uint16)

t = torch.from_numpy(f).cuda()
a = torch.tensor(float(A), dtype=torch.float32, device="cuda")
c = torch.tensor(float(C), dtype=torch.float32, device="cuda")
inner = c * t * (1.0 + a * t * t)
dev = (0.5 * t * (1.0 + torch.tanh(inner))).cpu().numpy()
dev16 = dev.astype(np.float16).view(np.uint16)

diff = fin & (host16 != dev16)
idx = np.nonzero(diff)[0]
print(f"gelu_probe: {int(fin.sum())} finite f16 inputs, {idx.size} device f16 results differ from the host table")
tanh_h = np.tanh(C * f * (ONE + A * f * f))
tanh_d = torch.tanh(inner).cpu().numpy()
tdiff = fin & (tanh_h.view(np.uint32) != tanh_d.view(np.uint32))
print(f"gelu_probe: tanhf differs (any ulp) for {int(tdiff.sum())} inputs; "
      f"max |ulp| {int(np.max(np.abs(tanh_h.view(np.int32)[fin].astype(np.int64) - tanh_d.view(np.int32)[fin]))) if fin.any() else 0}")
for i in idx[:40]:
    print(f"  x=0x{i:04x} ({f[i]:+.6g}): table 0x{host16[i]:04x} device 0x{dev16[i]:04x}")
