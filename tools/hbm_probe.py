"""HBM read / write / copy rates on this box (torch kernels, HIP events), 2 GiB buffers."""
import torch

dev = torch.device("cuda", 0)
n = (2 << 30) // 4
a = torch.ones(n, device=dev)
b = torch.empty_like(a)


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


nb = n * 4
print({"read_GBps": round(nb / t(lambda: a.sum()) / 1e9, 1),
       "write_GBps": round(nb / t(lambda: b.fill_(2.0)) / 1e9, 1),
       "copy_GBps": round(2 * nb / t(lambda: b.copy_(a)) / 1e9, 1)})
