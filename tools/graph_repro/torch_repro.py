"""Torch-level HIP-graph repro for the DEBUG_CLR_GRAPH_PACKET_CAPTURE symptom.

The plain-HIP repro (repro.hip) replays correctly in both capture modes; the PPO update graph does
not with packet capture. This narrows it down op by op: each case captures a small torch graph,
then replays it 4 times with eager launches of the same ops on other tensors in between, and
compares every replay with the eager result. Run twice, with the variable 0 and 1 (it is read when
HIP initialises): bash tools/graph_repro/run_torch.sh
"""
import os
import sys

import torch


def case_elementwise():
    x = torch.randn(1 << 16, device="cuda")
    y = torch.empty_like(x)

    def f():
        y.copy_(x * 2.0 + 1.0)
    return f, lambda: x * 2.0 + 1.0, y, [x], lambda: (torch.randn(1 << 16, device="cuda") * 3.0 + 2.0)


def case_fused_adam():
    torch.manual_seed(0)
    ps = [torch.randn(256, 256, device="cuda", requires_grad=True) for _ in range(6)]
    for p in ps:
        p.grad = torch.randn_like(p)
    lr = torch.tensor(1e-3, device="cuda")
    opt = torch.optim.Adam(ps, lr=lr, fused=True, capturable=True)
    opt.step()  # state
    other = [torch.randn(256, 256, device="cuda", requires_grad=True) for _ in range(6)]
    for p in other:
        p.grad = torch.randn_like(p)
    opt2 = torch.optim.Adam(other, lr=torch.tensor(3e-3, device="cuda"), fused=True, capturable=True)
    snap = [p.detach().clone() for p in ps]
    st = [{k: v.clone() for k, v in opt.state[p].items()} for p in ps]

    def restore():
        with torch.no_grad():
            for p, v, s in zip(ps, snap, st):
                p.copy_(v)
                for k, t in s.items():
                    opt.state[p][k].copy_(t)

    def f():
        opt.step()

    def ref():
        restore()
        opt.step()
        out = torch.cat([p.detach().flatten() for p in ps]).clone()
        restore()
        return out
    flat = lambda: torch.cat([p.detach().flatten() for p in ps])  # noqa: E731
    return f, ref, flat, restore, lambda: opt2.step()


def run(name, build):
    f, ref, out, inputs, eager_other = build()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        f()  # warm-up on the side stream (torch.cuda.graph convention)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    if callable(inputs):
        inputs()
    with torch.cuda.graph(g):
        f()
    ok = True
    for r in range(4):
        expect = ref() if name == "fused_adam" else ref()
        if callable(inputs):
            inputs()
        g.replay()
        torch.cuda.synchronize()
        got = out() if callable(out) else out
        err = (got - expect).abs().max().item()
        ok &= err <= 1e-6 * (1 + expect.abs().max().item())
        print(f"  {name} replay {r}: max |replay - eager| {err:.3g}")
        for _ in range(16):
            eager_other()
        torch.cuda.synchronize()
    return ok


def main():
    mode = os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "(unset)")
    res = {n: run(n, b) for n, b in (("elementwise", case_elementwise), ("fused_adam", case_fused_adam))}
    print(f"DEBUG_CLR_GRAPH_PACKET_CAPTURE={mode}: " + ", ".join(f"{k} {'correct' if v else 'WRONG'}" for k, v in res.items()))
    return 0 if all(res.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
