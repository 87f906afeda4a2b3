"""Calibration: device-to-device copy rate (read + write bytes / time) on one MI355X for buffers
below and above the 256 MiB Infinity Cache, and a write-only fill -- the stream rates the
assembly's mixed gather + store traffic can be compared with.  usage: python tools/copy_bw.py"""
import torch

dev = torch.device("cuda:0")
for mb in (56, 112, 224, 450, 900):
    n = mb * (1 << 20) // 8
    a = torch.empty(n, dtype=torch.float64, device=dev).uniform_()
    b = torch.empty_like(a)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 20 * 1e-3
    e0.record()
    for _ in range(20):
        b.fill_(1.0)
    e1.record()
    torch.cuda.synchronize()
    tf = e0.elapsed_time(e1) / 20 * 1e-3
    print(f"{mb} MB each: copy {2 * n * 8 / t / 1e12:.2f} TB/s (read+write), "
          f"fill {n * 8 / tf / 1e12:.2f} TB/s", flush=True)
    del a, b
