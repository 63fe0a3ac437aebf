"""Which rollout ops capture under a HIP graph on this torch/ROCm (diagnostic)."""
import torch, traceback
dev = "cuda"
def tryit(name, fn):
    torch.cuda.synchronize()
    fn()  # warm-up
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            fn()
        g.replay(); torch.cuda.synchronize()
        print(name, "OK", flush=True)
    except Exception as e:
        print(name, "FAIL", type(e).__name__, str(e).splitlines()[0], flush=True)
        torch.cuda.synchronize()
x = torch.randn(4096, 23, device=dev)
lin = torch.nn.Linear(23, 128).to(dev)
mean = torch.zeros(4096, 6, device=dev); std = torch.ones(6, device=dev)
tryit("randn", lambda: torch.randn(4096, 6, device=dev))
tryit("normal(tensor,tensor)", lambda: torch.normal(mean, std.expand(4096, 6)))
tryit("normal_", lambda: torch.empty(4096, 6, device=dev).normal_())
tryit("linear", lambda: lin(x))
with torch.inference_mode():
    tryit("linear(inference)", lambda: lin(x))
    tryit("normal(inference)", lambda: torch.normal(mean, std.expand(4096, 6)))
    tryit("randn(inference)", lambda: torch.randn(4096, 6, device=dev))
