"""Minimal repro: capture (zero_grad, fwd, bwd, [clip], opt.step) for an MLP; check that a replay from
a restored snapshot gives the same params before and after intervening eager work."""
import sys, torch, torch.nn as nn
torch.manual_seed(0)
dev = "cuda:0"
variant = sys.argv[1]
class EwLinear(nn.Linear):
    def forward(self, x):
        return (x[:, :, None] * self.weight.t()[None]).sum(1) + self.bias
L = EwLinear if "nomm" in sys.argv else nn.Linear
net = nn.Sequential(L(23, 128), nn.ELU(), L(128, 128), nn.ELU(), L(128, 1)).to(dev)
lr = torch.tensor(1e-3, device=dev)
if variant == "fused":
    opt = torch.optim.Adam(net.parameters(), lr=lr, fused=True, capturable=True)
elif variant == "foreach":
    opt = torch.optim.Adam(net.parameters(), lr=lr, foreach=True, capturable=True)
else:
    opt = torch.optim.SGD(net.parameters(), lr=1e-3)
X = torch.randn(4096, 23, device=dev); Y = torch.randn(4096, 1, device=dev)
idx = torch.randperm(4096, device=dev)
def upd():
    for i in range(4):
        if "slice" in sys.argv:
            xb, yb = X[i * 1024:(i + 1) * 1024], Y[i * 1024:(i + 1) * 1024]
        else:
            b = idx[i * 1024:(i + 1) * 1024]
            xb, yb = X[b], Y[b]
        loss = (net(xb) - yb).pow(2).mean()
        opt.zero_grad(set_to_none=False)
        loss.backward()
        if "noclip" not in sys.argv:
            nn.utils.clip_grad_norm_(net.parameters(), 1.0)
        opt.step()
if "rocblas" in sys.argv:
    torch.backends.cuda.preferred_blas_library("cublas")
print("blas", torch.backends.cuda.preferred_blas_library())
upd()
g = torch.cuda.CUDAGraph()
if "fence" in sys.argv:
    torch.cuda.synchronize(); torch._C._cuda_clearCublasWorkspaces()
if "side" in sys.argv:
    st = torch.cuda.Stream(); st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        upd()
    torch.cuda.current_stream().wait_stream(st)
    with torch.cuda.graph(g, stream=st):
        upd()
else:
    with torch.cuda.graph(g):
        upd()
if "fence" in sys.argv:
    torch.cuda.synchronize(); torch._C._cuda_clearCublasWorkspaces()
ps = list(net.parameters())
def snap():
    return [p.detach().clone() for p in ps], [{k: v.clone() for k, v in opt.state[p].items()} for p in ps]
def restore(s):
    with torch.no_grad():
        for p, v, st in zip(ps, s[0], s[1]):
            p.copy_(v)
            for k, t in st.items(): opt.state[p][k].copy_(t)
cur = lambda: torch.cat([(p.grad if "nostep" in sys.argv else p).detach().flatten() for p in ps]).clone()
s = snap()
g.replay(); torch.cuda.synchronize(); a = cur()
restore(s); upd(); torch.cuda.synchronize(); e = cur()
print(variant, sys.argv[2:], "replay vs eager", float((a - e).abs().max()))
with torch.no_grad():
    for _ in range(3): net(torch.randn(8192, 23, device=dev))   # intervening eager forward
restore(s); g.replay(); torch.cuda.synchronize(); b = cur()
print(variant, sys.argv[2:], "replay after eager fwd vs first replay", float((a - b).abs().max()))
restore(s); upd(); upd(); restore(s); g.replay(); torch.cuda.synchronize(); c = cur()
print(variant, sys.argv[2:], "replay after eager updates vs first replay", float((a - c).abs().max()))
X.copy_(torch.randn_like(X)); s2 = snap(); restore(s2)
g.replay(); torch.cuda.synchronize(); d1 = cur(); restore(s2); upd(); torch.cuda.synchronize(); d2 = cur()
print(variant, sys.argv[2:], "new data: replay vs eager", float((d1 - d2).abs().max()))
