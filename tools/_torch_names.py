import torch
torch.backends.cuda.matmul.allow_tf32 = False
dev = "cuda"
for (m, n, k, tr) in [(18688, 2048, 512, "NT"), (2048, 512, 18688, "TN"), (18688, 512, 2048, "NN")]:
    if tr == "NT":
        A = torch.randn(m, k, device=dev); W = torch.randn(n, k, device=dev); f = lambda: torch.mm(A, W.t())
    elif tr == "NN":
        A = torch.randn(m, k, device=dev); W = torch.randn(k, n, device=dev); f = lambda: torch.mm(A, W)
    else:
        A = torch.randn(k, m, device=dev); X = torch.randn(k, n, device=dev); f = lambda: torch.mm(A.t(), X)
    for _ in range(3):
        f()
torch.cuda.synchronize()
