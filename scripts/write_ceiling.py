"""Diagnostic: HBM write ceiling on this GPU for the emit output's size."""
import torch, time
x = torch.empty((4096, 100000), dtype=torch.int32, device="cuda")
for name, fn in [("fill", lambda: x.fill_(7)), ("zero", lambda: x.zero_())]:
    for _ in range(3): fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): fn()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(name, f"{ms:.3f} ms", f"{x.numel()*4/ms/1e6:.0f} GB/s")
y = torch.empty_like(x)
for _ in range(3): y.copy_(x)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20): y.copy_(x)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print("copy", f"{ms:.3f} ms", f"{2*x.numel()*4/ms/1e6:.0f} GB/s (read+write)")
