"""Experiment (profiling only): this box's plain write / copy bandwidth (torch fill_ and
copy_ of 640 MB), to calibrate the observation builder's figures box to box."""
import torch
x = torch.empty(160 * 1024 * 1024, dtype=torch.float32, device="cuda")
y = torch.empty_like(x)
for name, fn in (("fill", lambda: x.fill_(1.0)), ("copy", lambda: y.copy_(x))):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        fn()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) / 20 * 1e3
    nbytes = x.numel() * 4 * (1 if name == "fill" else 2)
    print(f"{name}: {us:.1f} us per call, {nbytes / us / 1e6:.2f} TB/s")
