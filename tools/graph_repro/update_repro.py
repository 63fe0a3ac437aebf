"""Narrowing the DEBUG_CLR_GRAPH_PACKET_CAPTURE symptom to the pieces of the PPO update graph
(tests/test_ppo.py::test_gpu_update_graph_matches_eager fails with the variable at
1). Each case captures a small update on a side stream (torch.cuda.graph), then per round:
restore the inputs, replay, compare with the eager update from the same inputs, and run some eager
work in between (torch ops, or the zbot env step, a kernel of another code object with a 1.7 KB
kernel-argument struct). Run once per capture mode (fresh processes):

    DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 python tools/graph_repro/update_repro.py
    DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 python tools/graph_repro/update_repro.py
"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "1")
import torch  # noqa: E402


def mlp(seed, hidden=(256, 128)):
    torch.manual_seed(seed)
    layers, d = [], 23
    for h in hidden:
        layers += [torch.nn.Linear(d, h), torch.nn.ELU()]
        d = h
    return torch.nn.Sequential(*layers, torch.nn.Linear(d, 6)).cuda()


def nothing():
    pass


def make_case(opt_kind, clip, between, batch=4096, hidden=(256, 128)):
    net = mlp(0, hidden)
    x = torch.randn(batch, 23, device="cuda")
    y = torch.randn(batch, 6, device="cuda")
    lr = torch.tensor(1e-3, device="cuda")
    opt = torch.optim.Adam(net.parameters(), lr=lr, fused=True, capturable=True) if opt_kind == "adam" else None
    params = list(net.parameters())
    for p in params:
        p.grad = torch.zeros_like(p)

    def update():
        for p in params:
            p.grad.zero_()
        loss = ((net(x) - y) ** 2).mean()
        loss.backward()
        if clip:
            torch.nn.utils.clip_grad_norm_(params, 1.0)
        if opt is not None:
            opt.step()
        elif opt_kind == "sgd":
            with torch.no_grad():
                for p in params:
                    p.add_(p.grad, alpha=-1e-3)

    def snap():
        st = [{k: v.clone() for k, v in opt.state[p].items()} for p in params] if opt else []
        return [p.detach().clone() for p in params], st

    def restore(s):
        ps, st = s
        with torch.no_grad():
            for p, v in zip(params, ps):
                p.copy_(v)
            for p, d in zip(params, st):
                for k, t in d.items():
                    opt.state[p][k].copy_(t)

    if opt_kind in ("none", "grads"):  # compare the (clipped) gradients instead of the parameters
        flat = lambda: torch.cat([p.grad.detach().flatten() for p in params]).clone()  # noqa: E731
    else:
        flat = lambda: torch.cat([p.detach().flatten() for p in params]).clone()  # noqa: E731
    return update, snap, restore, flat, x, between


def eager_torch():
    a = torch.randn(1 << 18, device="cuda")
    for _ in range(8):
        a = torch.tanh(a * 1.01 + 0.5)
    m = mlp(1)
    with torch.no_grad():
        m(torch.randn(2048, 23, device="cuda"))


_env = None


def eager_zbot():
    global _env
    import zbot_lab_amd
    if _env is None:
        cfg = zbot_lab_amd.tasks.load_cfg("zbot-6b-walking-v2")
        cfg.scene.num_envs = 512
        _env = zbot_lab_amd.make("zbot-6b-walking-v2", cfg=cfg)
        _env.reset()
    for _ in range(8):
        _env.step(torch.randn(512, 6, device="cuda"))


def run(name, opt_kind, clip, between, batch=4096, hidden=(256, 128)):
    update, snap, restore, flat, x, between_fn = make_case(opt_kind, clip, between, batch, hidden)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        update()  # warm-up on the side stream
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        update()
    ok = True
    for r in range(6):
        x.normal_()
        s0 = snap()
        update()
        torch.cuda.synchronize()
        expect = flat()
        restore(s0)
        g.replay()
        torch.cuda.synchronize()
        got = flat()
        err = (got - expect).abs().max().item()
        good = err <= 1e-5 * (1 + expect.abs().max().item())
        ok &= good
        print(f"  {name} round {r}: max |replay - eager| {err:.3g}{'' if good else '  <-- WRONG'}")
        between_fn()
        torch.cuda.synchronize()
    return ok


def main():
    mode = os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE")
    cases = [("sgd, torch between", "sgd", False, eager_torch), ("adam, torch between", "adam", False, eager_torch),
             ("adam+clip, torch between", "adam", True, eager_torch),
             ("adam+clip, nothing between", "adam", True, nothing),
             ("sgd+clip, torch between", "sgd", True, eager_torch),
             ("clip only (gradients), torch between", "none", True, eager_torch),
             ("clip only (gradients), nothing between", "none", True, nothing),
             ("sgd, zbot step between", "sgd", False, eager_zbot), ("adam+clip, zbot step between", "adam", True, eager_zbot)]
    cases += [("backward only (gradients), nothing between", "grads", False, nothing),
              ("backward only, batch 256", "grads", False, nothing, 256),
              ("backward only, hidden 64", "grads", False, nothing, 4096, (64,)),
              ("backward only, hidden 256x128, batch 1024", "grads", False, nothing, 1024),
              ("clip only, batch 256", "none", True, nothing, 256)]
    if os.environ.get("ONLY_NEW"):
        cases = cases[-5:]
    res = {}
    for name, o, c, b, *extra in cases:
        res[name] = run(name, o, c, b, *extra)
    print(f"DEBUG_CLR_GRAPH_PACKET_CAPTURE={mode}: " + "; ".join(f"{k}: {'correct' if v else 'WRONG'}" for k, v in res.items()))
    return 0


if __name__ == "__main__":
    sys.exit(main())
