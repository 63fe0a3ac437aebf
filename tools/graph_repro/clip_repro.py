"""The packet-capture symptom narrowed. Result (clip_repro_pc1.out / _pc0.out): with
DEBUG_CLR_GRAPH_PACKET_CAPTURE=1, a captured GEMM of 1024x512 with K = 8192 followed by a reduction
over its output (torch.sum or torch.linalg.vector_norm) replays wrong from the second replay on
(relative errors 1e-4 .. 1e2), with no eager work between replays; the same GEMM followed by an
elementwise op, smaller GEMMs followed by the same reductions, the reductions alone, foreach norms,
clip_grad_norm_ on static tensors and a small backward + clip all replay correctly, and every case
is correct with the variable at 0. The plain-HIP producer -> memset -> consumer graph replays
correctly in both modes (memset_repro.hip). In the PPO update the weight-gradient GEMMs of a
4096-sample minibatch feed clip_grad_norm_'s norm: update_repro.py ("clip only") fails the same way.
So the symptom is inside the ROCm runtime / library stack (a captured library GEMM and a dependent
reduction under packet capture), not a stale kernel argument of this code: zbot_lab_amd keeps
packet capture off (its kernels are not involved: update_repro.py fails with no zbot launch).

Each case captures one computation over static input tensors, refills the inputs with new values
before every replay and compares the replay with the eager computation.
Each case captures one piece of clip_grad_norm_ over static input tensors shaped like the PPO
MLP's gradients, refills the inputs with new values before every replay and compares the replay
with the eager computation. Run per capture mode (fresh processes):

    DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 python tools/graph_repro/clip_repro.py
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python tools/graph_repro/clip_repro.py
"""
import os
import sys

os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "1")
import torch  # noqa: E402

SHAPES = [(256, 23), (256,), (128, 256), (128,), (6, 128), (6,)]


def cases(g):
    def foreach_norm():
        return torch.stack(torch._foreach_norm(g, 2.0))

    def total_norm():
        return torch.linalg.vector_norm(torch.stack(torch._foreach_norm(g, 2.0)), 2.0).reshape(1)

    def vector_norm_big():
        return torch.linalg.vector_norm(g[2], 2.0).reshape(1)

    def sum_big():
        return g[2].sum().reshape(1)

    def stack_small():
        return torch.stack([t.sum() for t in g])

    def clip_coef_mul():
        tn = torch.linalg.vector_norm(torch.stack(torch._foreach_norm(g, 2.0)), 2.0)
        coef = torch.clamp(1.0 / (tn + 1e-6), max=1.0)
        out = torch._foreach_mul(g, coef)
        return torch.cat([t.flatten() for t in out])

    ws = [torch.nn.Parameter(torch.zeros_like(t)) for t in g]
    for w in ws:
        w.grad = torch.zeros_like(w)

    def clip_grad_norm_static():  # torch.nn.utils.clip_grad_norm_ on .grad copies of the inputs
        for w, t in zip(ws, g):
            w.grad.copy_(t)
        torch.nn.utils.clip_grad_norm_(ws, 1.0)
        return torch.cat([w.grad.flatten() for w in ws])

    def inplace_clip():  # its steps by hand, _foreach_mul_ in place
        h = [t.clone() for t in g]
        tn = torch.linalg.vector_norm(torch.stack(torch._foreach_norm(h, 2.0)), 2.0)
        coef = torch.clamp(1.0 / (tn + 1e-6), max=1.0)
        torch._foreach_mul_(h, coef)
        return torch.cat([t.flatten() for t in h])

    net = torch.nn.Sequential(torch.nn.Linear(23, 64), torch.nn.ELU(), torch.nn.Linear(64, 6)).cuda()
    x = g[0][:, :23].contiguous() if g[0].dim() == 2 else None
    for prm in net.parameters():
        prm.grad = torch.zeros_like(prm)

    def backward_norm():  # autograd backward, then the gradients' norms (no clipping)
        for prm in net.parameters():
            prm.grad.zero_()
        (net(g[0][:, :23]) ** 2).mean().backward()
        return torch.stack(torch._foreach_norm([prm.grad for prm in net.parameters()], 2.0))

    def backward_clip():  # autograd backward, then clip_grad_norm_
        for prm in net.parameters():
            prm.grad.zero_()
        (net(g[0][:, :23]) ** 2).mean().backward()
        torch.nn.utils.clip_grad_norm_(list(net.parameters()), 1.0)
        return torch.cat([prm.grad.flatten() for prm in net.parameters()])

    big_a = torch.randn(4096, 23, device="cuda")
    big_b = torch.randn(4096, 256, device="cuda")
    big_c = torch.randn(4096, 128, device="cuda")
    EXTRA.extend([big_a, big_b, big_c])

    def gemm_tall_k():  # the weight-gradient GEMM shape of a 4096-sample minibatch: K = 4096
        return torch.mm(big_b.t(), big_a).flatten()

    def gemm_tall_k_256x128():
        return torch.mm(big_c.t(), big_b).flatten()

    def gemm_small_k():
        return torch.mm(big_b[:256].t(), big_a[:256]).flatten()

    big_d = torch.randn(8192, 1024, device="cuda")
    big_e = torch.randn(8192, 512, device="cuda")
    EXTRA.extend([big_d, big_e])

    def gemm_then_norm():  # a dependent reduction right after the weight-gradient GEMM
        return torch.linalg.vector_norm(torch.mm(big_b.t(), big_a)).reshape(1)

    def big_gemm_then_norm():  # a slower GEMM (1024x512, K = 8192), then its norm
        return torch.linalg.vector_norm(torch.mm(big_d.t(), big_e)).reshape(1)

    def big_gemm_then_sum():
        return torch.mm(big_d.t(), big_e).sum().reshape(1)

    def big_gemm_then_scale():  # elementwise consumer
        return (torch.mm(big_d.t(), big_e) * 0.5).flatten()

    return [("GEMM 256x23 K=4096 -> vector_norm", gemm_then_norm), ("GEMM 1024x512 K=8192 -> vector_norm", big_gemm_then_norm),
            ("GEMM 1024x512 K=8192 -> sum", big_gemm_then_sum), ("GEMM 1024x512 K=8192 -> x0.5", big_gemm_then_scale),
            ("GEMM 256x23, K=4096 (weight gradient)", gemm_tall_k), ("GEMM 128x256, K=4096", gemm_tall_k_256x128),
            ("GEMM 256x23, K=256", gemm_small_k),
            ("clip_grad_norm_ on static grads", clip_grad_norm_static), ("clip by hand, in place", inplace_clip),
            ("backward + _foreach_norm", backward_norm), ("backward + clip_grad_norm_", backward_clip),
            ("_foreach_norm", foreach_norm), ("vector_norm(stack(_foreach_norm))", total_norm),
            ("vector_norm(one 128x256 tensor)", vector_norm_big), ("sum(one 128x256 tensor)", sum_big),
            ("stack of 6 sums", stack_small), ("clip: norms, coef, _foreach_mul", clip_coef_mul)]


EXTRA = []


def run(name, fn, g):
    out = torch.zeros(1, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = fn()
    ok = True
    errs = []
    for r in range(5):
        for t in g + EXTRA:
            t.normal_()
        expect = fn().clone()
        graph.replay()
        torch.cuda.synchronize()
        err = (out - expect).abs().max().item() / (1e-6 + expect.abs().max().item())
        errs.append(err)
        ok &= err <= 1e-5
    print(f"  {name}: relative errors per replay " + " ".join(f"{e:.2g}" for e in errs) + ("" if ok else "  <-- WRONG"))
    return ok


def main():
    torch.manual_seed(0)
    g = [torch.randn(sh, device="cuda") for sh in SHAPES]
    res = {n: run(n, f, g) for n, f in cases(g)}
    print(f"DEBUG_CLR_GRAPH_PACKET_CAPTURE={os.environ.get('DEBUG_CLR_GRAPH_PACKET_CAPTURE')}: "
          + "; ".join(f"{k}: {'correct' if v else 'WRONG'}" for k, v in res.items()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
