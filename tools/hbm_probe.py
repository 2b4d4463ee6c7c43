"""HBM write / copy throughput probes (torch fill_ / copy_ and a bf16 cast) to price the write-heavy GEMMs."""
import torch


def t(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / it / 1e3


n = 401408 * 384
a = torch.empty(n, dtype=torch.bfloat16, device="cuda")
b = torch.empty(n, dtype=torch.bfloat16, device="cuda")
c = torch.empty(n // 4, dtype=torch.bfloat16, device="cuda")
print(f"fill  {n * 2 / t(lambda: a.fill_(1.0)) / 1e12:.2f} TB/s (write only, {n * 2 / 1e6:.0f} MB)")
print(f"copy  {n * 4 / t(lambda: a.copy_(b)) / 1e12:.2f} TB/s (read + write)")
print(f"small-read big-write {n * 2.5 / t(lambda: a.view(-1, 4).copy_(c.view(-1, 1).expand(-1, 4))) / 1e12:.2f} TB/s")
# write-heavy mixes of the stage-1 GELU Linear: read 77 MB, write 2 x 308 MB
x = torch.empty(401408 * 96, dtype=torch.bfloat16, device="cuda")
print(f"fill x2 {2 * n * 2 / t(lambda: (a.fill_(1.0), b.fill_(2.0))) / 1e12:.2f} TB/s (two write-only streams)")
print(f"read 77 MB + write 2 x 308 MB (expand) {(n * 4 + x.numel() * 2) / t(lambda: (a.view(-1, 4).copy_(x.view(-1, 1).expand(-1, 4)), b.view(-1, 4).copy_(x.view(-1, 1).expand(-1, 4)))) / 1e12:.2f} TB/s")
