"""Time the training path's GEMM shapes (sa1 of SSG B=32: M = 524288 rows) with torch.mm vs a
chunked bmm (split-K by hand) for the tall-skinny dW = dY^T X."""
import torch
M = 32 * 512 * 32
def t(f, k=10):
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / k * 1e3
for cin, cout in ((3, 64), (64, 64), (64, 128), (131, 128), (128, 256)):
    Mx = M if cin < 100 else 32 * 128 * 64
    X = torch.randn(Mx, cin, device="cuda"); dY = torch.randn(Mx, cout, device="cuda")
    W = torch.randn(cout, cin, device="cuda"); b = torch.randn(cout, device="cuda")
    r = {"fwd addmm": t(lambda: torch.addmm(b, X, W.t())),
         "dW mm": t(lambda: torch.mm(dY.t(), X)),
         "dX mm": t(lambda: torch.mm(dY, W))}
    for ch in (2048, 8192):
        n = Mx // ch
        r["dW bmm%d" % ch] = t(lambda: torch.bmm(dY.view(n, ch, cout).transpose(1, 2), X.view(n, ch, cin)).sum(0))
    print(cin, cout, Mx, {k: round(v, 1) for k, v in r.items()})
