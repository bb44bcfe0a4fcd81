"""Bandwidth probes on the GPU box: what the HBM does for streams shaped like
the FK+J workload (read 8 rows, write 60 rows of N fp32), measured with the
same event timing as bench.py.  Reference points for the roofline discussion."""
import json
import sys
import torch

N = 1 << 20
dev = torch.device("cuda", 0)
q = torch.rand((8, N), device=dev)
out = torch.empty((60, N), device=dev)
big_in = torch.rand((16, N), device=dev)
big_out = torch.empty((16, N), device=dev)


def t(fn, k=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(k):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / k / 1e3


res = {}
s = t(lambda: out.fill_(1.0))
res["fill_60xN_f32_GBs"] = 60 * N * 4 / s / 1e9
s = t(lambda: big_out.copy_(big_in))
res["copy_16xN_f32_GBs"] = 2 * 16 * N * 4 / s / 1e9
s = t(lambda: torch.sum(big_in))
res["read_16xN_f32_GBs"] = 16 * N * 4 / s / 1e9
s = t(lambda: out[:8].copy_(q))
res["copy_8xN_f32_GBs"] = 2 * 8 * N * 4 / s / 1e9
print(json.dumps(res))
