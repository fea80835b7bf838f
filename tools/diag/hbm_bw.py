import torch, time
n = 515_000_000
x = torch.randn(n, device="cuda"); y = torch.empty_like(x)
for name, fn, byts in (("copy 1R1W", lambda: y.copy_(x), 8 * n), ("add 2R1W", lambda: torch.add(x, y, out=y), 12 * n),
                       ("fill 1W", lambda: y.fill_(1.0), 4 * n), ("sum 1R", lambda: x.sum(), 4 * n)):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(10): fn()
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 10
    print(f"{name:10s} {dt*1e3:8.3f} ms {byts/dt/1e12:6.2f} TB/s")
