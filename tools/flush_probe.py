"""Does a read flush evict the Infinity Cache?  Time a 200 MB streaming read (torch.sum) warm, after a 1 GiB read of an
unrelated buffer, and after a 1 GiB write of it (HIP events, median of 9)."""
import torch

a = torch.rand(50_000_000, device="cuda")  # 200 MB
f = torch.ones(268_435_456, device="cuda")  # 1 GiB


def t(pre):
    ts = []
    for _ in range(9):
        pre()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        a.sum()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return sorted(ts)[4]


for name, pre in (("warm", lambda: None), ("read_flush", lambda: f.sum()), ("write_flush", lambda: f.fill_(2.0)),
                  ("warm", lambda: None)):
    us = t(pre)
    print(f"{name:12s} 200 MB sum: {us:7.1f} us  ({200e6 / us / 1e6:.2f} TB/s)", flush=True)
